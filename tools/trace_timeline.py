"""Print the kernel timeline (duration, gap to the previous kernel) of the
last N dispatches of a rocprofv3 --kernel-trace CSV.
Usage: python tools/trace_timeline.py <dir with *kernel_trace.csv> [N]"""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))[-n:]
prev = None
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    kn = r["Kernel_Name"]
    import re
    m = re.search(r"(\w+_kernel(?:<[^>]*>)?|__amd_rocclr_\w+)", kn)
    name = m.group(1) if m else kn[:48]
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:6.1f}  {name}")
    prev = e
print(f"total {(int(rows[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")

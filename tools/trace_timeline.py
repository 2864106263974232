"""Timeline of a rocprofv3 kernel trace (CSV): start, duration, gap to the
previous kernel's end, queue, kernel, grid -- the last N dispatches.
Usage: python tools/trace_timeline.py <kernel_trace.csv> [N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("cda::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    gap = (s - end) / 1e3 if end is not None else 0.0
    print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  q{r['Queue_Id']}  {name[:40]:40s} "
          f"grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}")
    end = e if end is None else max(end, e)

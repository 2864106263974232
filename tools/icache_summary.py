"""Per-kernel sums of the counters collected by tools/icache_probe.sh.
usage: python tools/icache_summary.py gpurun_out/icache"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(set)
for sub in ("ic", "sq"):
    for f in glob.glob(f"{d}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(\w+_kernel(<\d+>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:32]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for k, c in sorted(acc.items(), key=lambda x: -x[1].get("SQ_WAVE_CYCLES", 0)):
    L = max(1, len(n[k]) // 2)
    hit, miss = c.get("SQC_ICACHE_HITS", 0), c.get("SQC_ICACHE_MISSES", 0)
    wc = c.get("SQ_WAVE_CYCLES", 0)
    print(f"{k:34s} launches~{L:3d} icache miss {miss / max(1, hit + miss):.4f} (dup {c.get('SQC_ICACHE_MISSES_DUPLICATE', 0) / max(1, hit + miss):.4f})"
          f"  wait_inst/wave_cycles {c.get('SQ_WAIT_INST_ANY', 0) / max(1, wc):.3f}  wait_any/wave_cycles {c.get('SQ_WAIT_ANY', 0) / max(1, wc):.3f}"
          f"  ifetch/launch {c.get('SQ_IFETCH', 0) / L:.3g}")

#!/bin/bash
# GPU-box A/B of the leaf kernel's namespace handling (round 5): the product
# (namespace kept in LDS from the first chunk, push-order check at the first
# chunk) against the same source built with -DCDA_LEAF_NS_RELOAD (namespace
# and neighbours' namespaces reloaded from global memory after the ninth
# block; build_var/nsreload).  The GPU suite first, then interleaved default
# benches (config 4, 1024 squares per step), then FETCH_SIZE / WRITE_SIZE
# passes of each over a short default bench: per-dispatch leaf_kernel bytes.
# Output: gpurun_out/<tag>/.
set -o pipefail
TAG=${1:?tag}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
lib() { [ "$1" = new ] && echo "$R/celestia-app_amd/libcda.so" || echo "$R/celestia-app_amd/build_var/nsreload/libcda.so"; }
for rep in 1 2 3; do
  for v in new reload; do
    CDA_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 20 \
      > "$OUT/ab_${v}_r${rep}.log" 2>&1 || exit $?
    python - "$OUT/ab_${v}_r${rep}.log" "$v" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(sys.argv[2], "sq/s %.1f" % j["value"], "ms/step %.3f" % j["ms_per_step"],
      {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
  done
done
cd /tmp && export TMPDIR=/tmp
for v in new reload; do
  for c in FETCH_SIZE WRITE_SIZE; do
    CDA_LIB=$(lib $v) timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${v}_$c" -o run \
      -- python3 "$R/bench.py" --no-cpu --no-extras --steps 2 --warmup 1 > "$OUT/pmc_${v}_$c.log" 2>&1 || exit $?
  done
done
cd "$R" && python3 - "$OUT" <<'PY' | tee -a "$OUT/ab.txt"
import csv, glob, sys, collections
out = sys.argv[1]
for v in ("new", "reload"):
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = collections.defaultdict(list)
        for f in glob.glob(f"{out}/pmc_{v}_{c}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if "leaf_kernel" in row["Kernel_Name"] and row["Counter_Name"] == c:
                    vals[row.get("Dispatch_Id", len(vals))].append(float(row["Counter_Value"]))
        per = [sum(x) for x in vals.values()]
        print(v, c, "leaf_kernel dispatches", len(per), "mean KiB %.0f" % (sum(per) / max(1, len(per))))
PY

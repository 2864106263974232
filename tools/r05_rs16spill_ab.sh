#!/bin/bash
# GPU-box A/B of the GF(2^16) encoder with lane-derived values recomputed from
# the thread id (round 5; the product: once per exchange call and per butterfly
# phase -- k = 512 13 -> 0 spilled values, k = 256 35 -> 22) against
# build_var/prev (the same source before).  (r05w ran a first form that
# recomputed them at every use: 0 spills, but +14 % VALU instructions.)
# GF(2^16) GPU tests first, interleaved benches at k = 512 batch 1 / 4 / 16 and
# k = 256 batch 1 / 4, then FETCH_SIZE / WRITE_SIZE of rs16_bs_kernel<9> per
# dispatch for each.  Output: gpurun_out/<tag>/.
set -o pipefail
TAG=${1:?tag}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "512 or 256 or gf16 or codec or split or linear or repair or fault" > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
lib() { [ "$1" = new ] && echo "$R/celestia-app_amd/libcda.so" || echo "$R/celestia-app_amd/build_var/prev/libcda.so"; }
for rep in 1 2 3; do
  for v in new prev; do
    for cfg in "512 1" "512 4" "512 16" "256 1" "256 4"; do
      set -- $cfg
      CDA_LIB=$(lib $v) timeout -k 10 200 python -u bench.py --k $1 --batch $2 --no-cpu --no-extras --steps 30 --warmup 40 \
        > "$OUT/ab_${v}_k$1_b$2_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_k$1_b$2_r${rep}.log" "$v" "$1" "$2" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
b = int(sys.argv[4])
rs = sum(st[x]["avg_ms"] for x in ("rs_q0", "rs_q3") if x in st)
print(sys.argv[2], "k", sys.argv[3], "batch", b, "ms/sq %.4f" % (j["ms_per_step"] / b), "RS/sq %.4f" % (rs / b),
      {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for v in new prev; do
  for c in FETCH_SIZE WRITE_SIZE; do
    CDA_LIB=$(lib $v) timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${v}_$c" -o run \
      -- python3 "$R/bench.py" --k 512 --batch 1 --distinct 1 --no-cpu --no-extras --steps 4 --warmup 1 \
      > "$OUT/pmc_${v}_$c.log" 2>&1 || exit $?
  done
done
cd "$R" && python3 - "$OUT" <<'PY' | tee -a "$OUT/ab.txt"
import csv, glob, sys, collections
out = sys.argv[1]
for v in ("new", "prev"):
    tot = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = collections.defaultdict(float)
        for f in glob.glob(f"{out}/pmc_{v}_{c}/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                if "rs16_bs_kernel" in row["Kernel_Name"] and row["Counter_Name"] == c:
                    vals[row.get("Dispatch_Id")] += float(row["Counter_Value"])
        tot[c] = sum(vals.values()) / max(1, len(vals))
        print(v, c, "rs16_bs_kernel dispatches", len(vals), "mean KiB %.0f" % tot[c])
    # gfx950: HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) KiB, two launches per square
    print(v, "MB per square (2 launches, 2xFETCH+WRITE) %.1f" % (2 * (2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024 / 1e6))
PY

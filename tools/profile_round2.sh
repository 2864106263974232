#!/bin/bash
# Round evidence in one GPU call (run via gpurun): rocprofv3 kernel stats and
# separate PMC passes of the k=128 bench (config 4 shard) and of a k=512 batch
# (config 3, GF(2^16)), merged into one summary, then the full bench line with
# that summary.  Usage: tools/profile_round2.sh <tag>  -> gpurun_out/prof_<tag>*
set -o pipefail
TAG=${1:-r02d}
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp
for K in 128 512; do
  OUT=$R/gpurun_out/prof_${TAG}_k$K
  mkdir -p $OUT
  if [ $K = 128 ]; then B="$R/bench.py --no-cpu --no-extras"; else B="$R/bench.py --k 512 --batch 1 --distinct 1 --no-cpu --no-extras --steps 4 --warmup 1"; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1 || exit 2
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1 || exit 3
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1 || exit 4
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/wait -o run -- python3 $B > $OUT/wait.log 2>&1 || exit 5
  cd $R && python3 tools/pmc_summary.py $OUT $OUT/pmc.json > $OUT/pmc_summary.log 2>&1 || exit 6
  cd /tmp
done
cd $R
python3 - "$R/gpurun_out/prof_${TAG}_k128/pmc.json" "$R/gpurun_out/prof_${TAG}_k512/pmc.json" "$R/gpurun_out/${TAG}_pmc.json" <<'PY' || exit 7
import json, sys
a = json.load(open(sys.argv[1])); b = json.load(open(sys.argv[2]))
for k, v in b.items():          # the GF(2^16) encoder and any kernel only k=512 runs
    if k not in a:
        a[k] = v
a["_note"] = "k=128 bench (--no-extras) PMC passes; kernels absent there (rs_gf16) from single k=512 squares (bench.py reads rs_gf16 per launch x 2 launches as one square)"
json.dump(a, open(sys.argv[3], "w"), indent=1)
PY
CDA_PMC_SUMMARY=$R/gpurun_out/${TAG}_pmc.json timeout -k 10 400 python3 -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 8
tail -c 600 gpurun_out/${TAG}_bench.json
echo done

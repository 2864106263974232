# r04x: effective clock and wait fractions of the hash kernels at 128 vs 1024
# squares per step (config 4's N = 8 vs N = 1 shard): one SQ pass + the
# kernel trace for each, summarised per kernel by tools/pmc_summary3.py
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for b in 128 1024; do
  OUT=$R/gpurun_out/r04x_b$b; rm -rf $OUT; mkdir -p $OUT
  B="$R/bench.py --batch $b --no-cpu --no-extras --steps 3 --warmup 1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/wait -o run -- python3 $B > $OUT/wait.log 2>&1
  cd $R && python3 tools/pmc_summary3.py $OUT $R/gpurun_out/r04x_b${b}_pmc.json 128 7 $b "python3 bench.py --batch $b" > $OUT/sum.log 2>&1; cd /tmp
done
cd $R && python3 - <<'PY'
import json
for b in (128, 1024):
    d = json.load(open(f"gpurun_out/r04x_b{b}_pmc.json"))
    for k in ("nmt_leaves", "nmt_levels", "rs_gf8_bs"):
        v = d.get(k, {})
        print(b, k, "avg_us", round(v.get("avg_us", 0), 1), "clock", round(v.get("effective_clock_ghz") or 0, 3),
              "wait_any", round(v.get("wait_any_frac") or 0, 3), "valu/wave", round(v.get("valu_insts_per_wave") or 0))
PY

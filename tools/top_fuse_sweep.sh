#!/bin/bash
# Batch headline vs the level at which the NMT trees switch to the fused
# tree-top kernel (CDA_TOP_FUSE = nodes per tree; auto = never for a batch of 128).
set -o pipefail
mkdir -p gpurun_out/topfuse
for r in 1 2; do for f in ${FUSE_LIST:-auto 8 16 32 64}; do
  if [ $f = auto ]; then unset CDA_TOP_FUSE; else export CDA_TOP_FUSE=$f; fi
  timeout -k 10 120 python bench.py --no-cpu --no-extras --steps ${STEPS:-20} > gpurun_out/topfuse/f$f.log 2>&1 || { tail -5 gpurun_out/topfuse/f$f.log; exit 1; }
  python - "$f" <<'PY'
import json, sys
t = sys.argv[1]
s = open(f"gpurun_out/topfuse/f{t}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("fuse", t, round(j["value"]), "sq/s", round(j["ms_per_step"], 3), "ms", {k: round(x["avg_ms"], 3) for k, x in j["stages"].items()}, "parity", j["parity"]["matched"], flush=True)
PY
done; done

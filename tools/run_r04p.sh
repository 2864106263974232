# r04p: instruction-fetch counters of the bitsliced GF(2^16) encoder (k=512,
# batch 4): product vs the wave-fold build (+17 % code, 15 % slower at batch 4)
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04p/prod bash tools/icache_probe.sh
CDA_LIB=$GRAFT_REPO_ROOT/celestia-app_amd/build_var/wfold/libcda.so OUT=$GRAFT_REPO_ROOT/gpurun_out/r04p/wfold bash tools/icache_probe.sh
python tools/icache_summary.py gpurun_out/r04p/prod | head -8
python tools/icache_summary.py gpurun_out/r04p/wfold | head -8

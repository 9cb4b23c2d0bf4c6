# Rank-block sweep time for the decompositions of 8192² on 4 and 8 ranks, item orders 0/3 (each config twice).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/decomp; mkdir -p $O
PROBE_CFG=8:rows,8:aspect,4:rows,4:aspect PROBE_ITERS=400 \
PROBE_ENV="PE_ORDER=0 PE_TI=8;PE_ORDER=3 PE_TI=16;PE_ORDER=3 PE_TI=12;PE_ORDER=0 PE_TI=8;PE_ORDER=3 PE_TI=16;PE_ORDER=3 PE_TI=12" \
  timeout -k 10 500 python3 tools/block_probe.py > $O/block.txt 2>&1; rc=$?; grep -v amdgpu $O/block.txt; exit $rc

set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/occ; mkdir -p $O
PROBE_CFG=8:aspect,2:aspect,1:aspect PROBE_ITERS=300 PROBE_ENV="PE_ORDER=3 PE_TI=16;PE_ORDER=3 PE_TI=16 PE_SKERNEL=4;PE_ORDER=3 PE_TI=16;PE_ORDER=3 PE_TI=16 PE_SKERNEL=4" \
  timeout -k 10 300 python3 tools/block_probe.py > $O/block.txt 2>&1

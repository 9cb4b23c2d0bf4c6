set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/stamps; mkdir -p $O
PROBE_CFG=8:aspect,1:aspect PROBE_ENV="PE_ORDER=3 PE_TI=16" timeout -k 10 200 python3 tools/stamp_probe.py > $O/stamps.txt 2>&1

# HBM roofline (stream2) + per-kernel times of multi-rank blocks (block_probe under rocprofv3).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r1b; mkdir -p $O
timeout -k 10 120 ./bin/stream2 > $O/stream2.txt 2>&1 || exit 1
export TMPDIR=/tmp
PROBE_CFG=8:aspect,4:aspect,2:aspect,1:aspect PROBE_ITERS=200 timeout -k 10 240 \
  rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 tools/block_probe.py > $O/block.txt 2>&1
echo EXIT $?

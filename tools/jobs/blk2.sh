#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/blk2
PROBE_CFG=8:aspect PROBE_ENV="PE_TI=8 PE_ORDER=0" PROBE_ITERS=400 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/blk2/prof -o run -- python3 $R/tools/block_probe.py > $R/gpurun_out/blk2/probe.log 2>&1
rc=$?
cat $R/gpurun_out/blk2/probe.log | tail -3
find $R/gpurun_out/blk2/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
exit $rc

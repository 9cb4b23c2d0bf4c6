# Round 5, twenty-sixth GPU call: the layouts' cost of a mixed (lane-tested)
# row step (PE_COST_MIXED, default 1.3 uniform steps) on the mid-size blocks.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5twentysixth; mkdir -p $O
cd $R
for rep in 1 2; do
  for cm in 1.0 1.3 1.6 2.0; do
    PE_COST_MIXED=$cm PROBE_CFG=8:device,8:4x2,4:device timeout -k 10 120 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/mixed $cm /"
    PE_COST_MIXED=$cm PROBE_GRID=2048x2048 PROBE_CFG=1:device timeout -k 10 100 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/mixed $cm /"
  done
done
echo EXIT 0

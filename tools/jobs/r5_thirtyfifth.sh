# Round 5, thirty-fifth GPU call: the row slabs' per-rank time with the halo-
# push kernel (PE_PUSH_LOOPBACK=1: pushes into its own receive buffer) against
# the plain kernel the projections used (8192^2 2 / 4 / 8 ranks, 16384^2 8).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirtyfifth; mkdir -p $O
cd $R
for rep in 1 2; do
  for lb in 0 1; do
    PE_PUSH_LOOPBACK=$lb PROBE_CFG=8:device,4:device,2:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/loopback $lb /"
  done
done
for lb in 0 1; do
  PE_PUSH_LOOPBACK=$lb PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_CFG=8:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/loopback $lb /"
done
echo EXIT 0

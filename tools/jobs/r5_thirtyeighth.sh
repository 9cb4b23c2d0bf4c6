# Round 5, thirty-eighth GPU call: the halo push's layout — boundary pieces cut
# off and dealt first (default) or the plain layout (PE_PUSH_FIRST=0) — with
# the push kernel (PE_PUSH_LOOPBACK=1), row slabs of 8192^2 and 16384^2.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirtyeighth; mkdir -p $O
cd $R
for rep in 1 2; do
  for pf in 1 0; do
    PE_PUSH_FIRST=$pf PE_PUSH_LOOPBACK=1 PROBE_CFG=8:device,4:device,2:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/first $pf /"
  done
done
for pf in 1 0; do
  PE_PUSH_FIRST=$pf PE_PUSH_LOOPBACK=1 PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_CFG=8:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/first $pf /"
done
echo EXIT 0

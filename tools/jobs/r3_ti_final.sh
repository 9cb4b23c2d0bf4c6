# Rows per item of the three-step sweep at 8192^2 and 16384^2 at HEAD (one placement per grid, tools/ti_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
PROBE_GRIDS=8192x8192 PROBE_TI=64,72,80,88,96,112 PROBE_ALGO=4 PROBE_ITERS=600 PROBE_REPS=3 timeout -k 10 300 python3 -u tools/ti_probe.py || exit 1
PROBE_GRIDS=16384x16384 PROBE_TI=64,80,96,128 PROBE_ALGO=4 PROBE_ITERS=150 PROBE_REPS=2 timeout -k 10 300 python3 -u tools/ti_probe.py || exit 1
echo EXIT 0

# Band-row cost weight on the large blocks at ONE memory placement (tools/layout_probe.py:
# one solver, re-laid out per configuration, rounds): 8192^2, the 2-rank 8192^2 block, 16384^2
# -> profiles/r2_gencost.txt (appended)
set -o pipefail
cd $GRAFT_REPO_ROOT
PROBE_GRID=8192x8192 PROBE_P=1 PROBE_ROUNDS=3 PROBE_CFGS="24s PE_GEN_COST=3;24s PE_GEN_COST=2;24s PE_GEN_COST=1.5" timeout -k 10 200 python3 -u tools/layout_probe.py || exit 1
PROBE_GRID=8192x8192 PROBE_P=2 PROBE_ROUNDS=3 PROBE_CFGS="24s PE_GEN_COST=3;24s PE_GEN_COST=2;24s PE_GEN_COST=1.5" timeout -k 10 200 python3 -u tools/layout_probe.py || exit 1
PROBE_GRID=16384x16384 PROBE_P=1 PROBE_ITERS=200 PROBE_ROUNDS=2 PROBE_CFGS="18d PE_GEN_COST=3;18d PE_GEN_COST=2;24s PE_GEN_COST=2;24s PE_GEN_COST=3" timeout -k 10 300 python3 -u tools/layout_probe.py || exit 1
echo EXIT 0

# Band-row cost weight of the static LPT layout (PE_GEN_COST) on every static block:
# 2400x3200, 1600x2400 (1 rank), the 8/4/2-rank 8192^2 blocks and 8192^2 itself -> profiles/r2_gencost.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
E="${GEN_ENV:-PE_GEN_COST=3;PE_GEN_COST=1.5;PE_GEN_COST=2;PE_GEN_COST=4.5;PE_GEN_COST=6;PE_GEN_COST=3}"
for g in 2400x3200 1600x2400; do
  PROBE_GRID=$g PROBE_CFG=1:device PROBE_ENV="$E" PROBE_ITERS=400 timeout -k 10 200 python3 -u tools/block_probe.py || exit 1
done
PROBE_CFG=${GEN_CFG:-8:device} PROBE_ENV="$E" PROBE_ITERS=300 timeout -k 10 400 python3 -u tools/block_probe.py || exit 1
echo EXIT 0

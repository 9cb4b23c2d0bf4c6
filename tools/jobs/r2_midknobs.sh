# Layout knobs on the mid-size static blocks (8-rank 8192^2 block, 2400x3200): heavy-item
# splitting off, fewer waves than the resident grid -> profiles/r2_midknobs.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
E="PE_GEN_COST=2;PE_HEAVY_SPLIT=0;PE_WAVES=1792;PE_WAVES=1536;PE_WAVES=1024;PE_GEN_COST=2"
PROBE_GRID=2400x3200 PROBE_CFG=1:device PROBE_ENV="$E" PROBE_ITERS=400 timeout -k 10 200 python3 -u tools/block_probe.py || exit 1
PROBE_CFG=8:device PROBE_ENV="$E" PROBE_ITERS=300 timeout -k 10 200 python3 -u tools/block_probe.py || exit 1
echo EXIT 0

# Per-rank load balance of the row-slab decompositions of 8192^2 (8 and 4 ranks, the
# bench's `device` default): every rank's block timed on one GPU (timing-only transport,
# eager, tuned rows per item) -> profiles/r2_rank_balance.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
PROBE_CFG=8:device,4:device,2:device PROBE_RANKS=all PROBE_ITERS=300 timeout -k 10 300 python3 -u tools/block_probe.py || exit 1
echo EXIT 0

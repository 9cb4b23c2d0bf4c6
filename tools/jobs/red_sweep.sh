# Reduction-kernel variants at 8192² (it/s, 2000 iterations, no tol): multi-block kRed with
# PE_REDBLOCKS blocks vs the single-workgroup kRed1 (PE_RED1_MAX above the item count).
set -o pipefail
cd $GRAFT_REPO_ROOT
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
run() { echo -n "$1: "; env $1 timeout -k 10 60 $BIN --json --quiet --max-iter 2000 --no-tol 8192 8192 | grep -o '"iters_per_s": [0-9.]*' || exit 1; }
for rep in 1 2; do
  run PE_REDBLOCKS=16; run PE_RED1_MAX=40000; run PE_REDBLOCKS=8; run PE_REDBLOCKS=32; run PE_REDBLOCKS=64
done

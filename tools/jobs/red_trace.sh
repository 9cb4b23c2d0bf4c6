# Reduction kernel duration at 8192²: multi-block kRed (default, 16 blocks) vs single-workgroup kRed1 (PE_RED1_MAX).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/redtr; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
cd /tmp && export TMPDIR=/tmp
for v in ${RED_VARIANTS:-"PE_REDBLOCKS=16" "PE_RED1_MAX=40000" "PE_REDBLOCKS=64" "PE_REDBLOCKS=4"}; do
  n=${v//=/_}
  env $v timeout -k 10 120 rocprofv3 --kernel-trace -d $O/$n -o run -- $BIN --json --quiet --max-iter 600 --no-tol 8192 8192 > $O/$n.log 2>&1 || exit 1
done
echo done

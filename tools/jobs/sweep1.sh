set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sweep1; mkdir -p $O
run() { timeout -k 10 100 ./bin/pe_hip --json --max-iter 300 --no-tol "$@" 8192 8192 2>&1 | grep '^{' ; }
( for o in 0 1; do for ti in 4 8 16 32; do for wv in 2048 4096 8192; do
   echo "order=$o ti=$ti waves=$wv $(PE_ORDER=$o PE_TI=$ti PE_WAVES=$wv run)" || exit 1; done; done; done ) > $O/res.txt 2>&1
echo EXIT $?

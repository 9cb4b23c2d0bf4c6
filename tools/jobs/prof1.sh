set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1
export TMPDIR=/tmp
( for v in 0 1; do for ti in 8 16 32 64; do echo "variant=$v ti=$ti"; PE_TI=$ti timeout -k 10 100 ./bin/pe_hip --json --variant $v --max-iter 400 --no-tol 8192 8192 || exit 1; done; done ) > gpurun_out/prof1/sweep.txt 2>&1 && \
timeout -k 10 200 ./bin/pe_hip --json --variant 1 8192 8192 > gpurun_out/prof1/v1_full.txt 2>&1 && \
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1/rp -o run -- $GRAFT_REPO_ROOT/bin/pe_hip --max-iter 300 4096 4096 > $GRAFT_REPO_ROOT/gpurun_out/prof1/rp.log 2>&1
echo EXIT $?

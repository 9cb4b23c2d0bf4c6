# Per-iteration fixed costs at the per-rank block sizes of the 2/4/8-GPU
# runs (1 GPU): iteration rate vs kernel time from a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/small; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
for g in "4097 8192" "4097 4097" "2049 4097" "2900 2900"; do echo "grid $g"; timeout -k 10 60 $BIN --json --quiet --max-iter 1000 --no-tol $g | grep -o '"iters_per_s": [0-9.]*' || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $BIN --quiet --max-iter 400 --no-tol 2049 4097 > $O/kt.log 2>&1
echo EXIT $?

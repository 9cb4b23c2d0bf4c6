# kRed batched-load check: it/s at 8192², steady-state kernel stats, determinism/golden GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/red; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
for i in 1 2 3; do timeout -k 10 60 $BIN --json --quiet --max-iter 2000 --no-tol 8192 8192 | grep -o '"iters_per_s": [0-9.]*' || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "golden or deterministic or orders or parity or fused or bench" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $BIN --quiet --max-iter 500 --no-tol 8192 8192 > $O/kt.log 2>&1
echo "rocprof rc=$?"

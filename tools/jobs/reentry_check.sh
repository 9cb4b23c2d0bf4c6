# Re-entry check on a fresh box: smoke(), GPU test suite, 1-GPU bench, kernel-trace stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/reentry; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo smoke failed; tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.txt 2> $O/bench.err; rc=$?
cat $O/bench.txt; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $GRAFT_REPO_ROOT/bin/pe_hip --quiet --max-iter 500 --no-tol 8192 8192 > $O/kt.log 2>&1
echo "rocprof rc=$?"

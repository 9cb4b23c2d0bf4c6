# Re-entry check: GPU test suite + 1-GPU bench on the freshly built tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/check; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.txt 2> $O/bench.err; rc=$?
cat $O/bench.txt; echo "bench rc=$rc"; exit $rc

# Full GPU test suite + short and long 1-GPU bench (regression check after a change).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/suite; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -5 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
cat $O/bench20.json
echo EXIT 0

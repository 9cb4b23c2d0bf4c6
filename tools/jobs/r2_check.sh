# Round 2: GPU test suite, then the small-grid profile (r2_small.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/check; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -15 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
bash tools/jobs/r2_small.sh

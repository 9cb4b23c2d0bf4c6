# Round 6, thirty-first GPU call: the cached layouts equal fresh ones (new
# layout tests).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirtyfirst; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_layout.py -m gpu -k "fresh_layout" > $O/t.txt 2>&1 || { tail -40 $O/t.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/t.txt
echo EXIT 0

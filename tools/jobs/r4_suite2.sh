# Round-4 GPU suite after the boundary-first fix of the equal-cost layout's
# round dealing (the overlap's kSignal variant counts list positions
# 0 .. nb-1 as boundary items) -> profiles/r4_suite.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4suite; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_layout.py -x -q --tb=short --timeout 200 --timeout-method thread > $O/layout.txt 2>&1 || { tail -30 $O/layout.txt; exit 1; }
tail -1 $O/layout.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 240 --timeout-method thread > $O/suite2.txt 2>&1 || { tail -30 $O/suite2.txt; exit 1; }
tail -2 $O/suite2.txt
echo EXIT 0

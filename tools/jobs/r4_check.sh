# Round 4 check at HEAD: layout / three-step / residual GPU tests, then the
# per-rank blocks of the 2/4/8-rank 8192^2 splits (tools/block_probe.py) with
# the default layouts -> profiles/r4_check.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --tb=short --timeout 240 --timeout-method thread tests/test_layout.py tests/test_three_step.py tests/test_residual.py > $O/r4_check_tests.txt 2>&1; rc=$?
tail -5 $O/r4_check_tests.txt
[ $rc -eq 0 ] || exit $rc
PROBE_CFG=8:device,4:device,2:device,8:4x2 timeout -k 10 300 python3 -u tools/block_probe.py > $O/r4_block.txt 2>&1 || { tail $O/r4_block.txt; exit 1; }
cat $O/r4_block.txt
echo EXIT 0

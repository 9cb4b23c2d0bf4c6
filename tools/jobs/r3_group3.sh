# Virtual-rank group driver with the three-step sweep: targeted GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=$GRAFT_REPO_ROOT/gpurun_out/group3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_three_step.py tests/test_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread \
  -k "three_step or virtual_ranks or thin_blocks or multi_process_2d" > $O/pytest.txt 2>&1; rc=$?
tail -8 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
echo EXIT 0

# Round 3: multi-process (one GPU) tests of the two-step row slabs: host-staged / P2P / push, bench, T_MPI.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3mp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -v --timeout 200 --timeout-method thread \
  -k "multi_process or halo_push or slow_rank or self_launch or two_process or stalled" > $O/pytest.txt 2>&1; rc=$?
tail -30 $O/pytest.txt
exit $rc

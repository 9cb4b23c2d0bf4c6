# Round 4 new / changed GPU tests only (residual check, random init, drift
# restart, resident late workgroup, alternating directions, transport
# diagnostics, 2-D three-step overlap, two-step odd counts) -> profiles/r4_new_tests.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --tb=short --timeout 240 --timeout-method thread \
  tests/test_residual.py tests/test_three_step.py::test_three_step_alternating_directions \
  "tests/test_gpu.py::test_resident_late_workgroup_restarts" "tests/test_gpu.py::test_resident_barrier_timeout_falls_back" \
  tests/test_gpu.py::test_bench_reports_transport_fallbacks tests/test_gpu.py::test_p2p_selftest_failure_falls_back \
  tests/test_gpu.py::test_halo_push_selftest_failure_falls_back tests/test_gpu.py::test_multi_process_2d_three_step \
  tests/test_two_step.py::test_two_step_rejects_odd_counts > $O/r4_new_tests.txt 2>&1; rc=$?
tail -30 $O/r4_new_tests.txt
exit $rc

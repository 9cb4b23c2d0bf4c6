# Round 6, twelfth GPU call: the halo-path choice on the live iteration (no
# reset per candidate, 1 + 3 sweeps): its construction cost (PE_CTOR_TRACE),
# the choice / bitwise tests, the host-staged default-path jobs.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twelfth; mkdir -p $O
cd $R
PROBE_CFG=8:rows,8:4x2,4:rows PE_CTOR_TRACE=1 timeout -k 10 300 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -30 $O/ctor.txt; exit 1; }
grep -E "halo path|construction" $O/ctor.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "halo_path_choice or loopback_transport_bitwise or multi_process_2d_host_staged or halo_put or diagnostic" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "PASSED|FAILED" $O/tests.txt
echo EXIT 0

# Multi-process (IPC / P2P) GPU tests first, then the whole GPU suite, then the occupancy probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/mp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "multi_process or two_process" > $O/mp.txt 2>&1; rc=$?
tail -12 $O/mp.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
PROBE_CFG=8:aspect,2:aspect,1:aspect PROBE_ITERS=300 PROBE_ENV="PE_ORDER=3 PE_TI=16;PE_ORDER=3 PE_TI=16 PE_SKERNEL=4;PE_ORDER=3 PE_TI=16;PE_ORDER=3 PE_TI=16 PE_SKERNEL=4" \
  timeout -k 10 300 python3 tools/block_probe.py > $O/occ.txt 2>&1; rc=$?; grep -v amdgpu $O/occ.txt; exit $rc

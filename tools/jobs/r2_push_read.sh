# Halo push without the import kernel (sweeps read halo rows from the receive buffers): multi-process push tests + checkpoint/resume.
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "multi_process or halo_push or checkpoint or two_process" 2>&1 | grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" | tail -40

set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gput2; mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_gpu.py -k "two_process" -x -q > $O/pytest.txt 2>&1; echo "rc=$?"; tail -30 $O/pytest.txt

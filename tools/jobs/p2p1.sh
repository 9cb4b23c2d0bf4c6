#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/p2p
timeout -k 10 500 python -m pytest tests/test_gpu.py -x -q -m gpu -k "multi_process" > gpurun_out/p2p/tests.log 2>&1
rc=$?
tail -30 gpurun_out/p2p/tests.log
exit $rc

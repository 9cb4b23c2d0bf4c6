#!/bin/bash
# overlap (single launch, counted boundary items, per-XCD writeback): tests + delay-transport probe
set -o pipefail
mkdir -p gpurun_out/ov3
timeout -k 10 400 python -m pytest tests/test_gpu.py -x -q -m gpu -k "multi_process or host_staged or virtual" > gpurun_out/ov3/tests.log 2>&1 || { tail -30 gpurun_out/ov3/tests.log; exit 1; }
tail -2 gpurun_out/ov3/tests.log
PROBE_GRAPH=0 PROBE_OV=0,1:8,1:8:2,1:0,1:16 PROBE_CFG=8:aspect,4:aspect,2:aspect timeout -k 10 300 python tools/overlap_probe.py 20 12 > gpurun_out/ov3/probe.log 2>&1
rc=$?
cat gpurun_out/ov3/probe.log
exit $rc

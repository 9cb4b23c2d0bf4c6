#!/bin/bash
# overlap v2 (single launch + signal): tests + probe
set -o pipefail
mkdir -p gpurun_out/ov2
timeout -k 10 400 python -m pytest tests/test_gpu.py -x -q -m gpu -k "overlap or multiproc or host_staged or virtual or golden" > gpurun_out/ov2/tests.log 2>&1 && \
PROBE_GRAPH=0 PROBE_OV=0,1:0,1:8,1:32 PROBE_CFG=2:aspect,8:aspect timeout -k 10 300 python tools/overlap_probe.py 20 12 > gpurun_out/ov2/probe.log 2>&1 && \
PROBE_GRAPH=1 PROBE_OV=0,1:8 PROBE_CFG=2:aspect,8:aspect timeout -k 10 200 python tools/overlap_probe.py 20 12 > gpurun_out/ov2/probe_graph.log 2>&1
rc=$?
tail -3 gpurun_out/ov2/tests.log; cat gpurun_out/ov2/probe*.log
exit $rc

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/blk1
PROBE_CFG=8:aspect,4:aspect PROBE_ENV="PE_TI=8;PE_TI=8 PE_WAVES=1024;PE_TI=8 PE_WAVES=1536;PE_TI=8 PE_SKERNEL=3;PE_TI=8 PE_WAVES=1024 PE_SKERNEL=3;PE_TI=6;PE_TI=10;PE_TI=8 PE_PAD=64;PE_TI=8 PE_PAD=256;PE_TI=8 PE_PAD=1024" timeout -k 10 400 python tools/block_probe.py > gpurun_out/blk1/probe2.log 2>&1
rc=$?
cat gpurun_out/blk1/probe2.log
exit $rc

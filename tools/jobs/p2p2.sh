#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/p2p
for n in 2 4 8; do
  PE_COMM=host PE_ALLREDUCE=p2p timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600+n)) tools/allreduce_latency.py >> gpurun_out/p2p/lat.log 2>gpurun_out/p2p/lat_err_$n.log || { tail -20 gpurun_out/p2p/lat_err_$n.log; exit 1; }
done
cat gpurun_out/p2p/lat.log

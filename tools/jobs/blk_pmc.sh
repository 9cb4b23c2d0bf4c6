#!/bin/bash
# PMC comparison of the P=8 block sweep at ti=8 (fast) vs ti=35 (slow, long items)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bpmc; mkdir -p $O
export PROBE_CFG=8:aspect PROBE_ITERS=60
for ti in 8 35; do
  export PROBE_ENV="PE_TI=$ti PE_ORDER=0"
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum -d $O/a$ti -o run -- python3 $R/tools/block_probe.py > $O/a$ti.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum -d $O/b$ti -o run -- python3 $R/tools/block_probe.py > $O/b$ti.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum -d $O/c$ti -o run -- python3 $R/tools/block_probe.py > $O/c$ti.log 2>&1 || exit 1
done
for f in $O/*/run_results.db; do echo "== $f"; python3 $R/tools/pmc_by_dispatch.py $f --kernel kS --group 1000; done

set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/apmc; mkdir -p $O
P="python3 $GRAFT_REPO_ROOT/tools/alloc_pmc.py 6"
timeout -k 10 240 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum -d $O/a -o run -- $P > $O/a.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum -d $O/b -o run -- $P > $O/b.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum -d $O/c -o run -- $P > $O/c.log 2>&1
echo EXIT $?

# Round profile set: kernel-trace stats and PMC counters of the single-sweep
# solver at 8192² (summaries copied into profiles/ afterwards).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/prof; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
ARGS="--quiet --max-iter 200 --no-tol 8192 8192"
for rb in 4 8 16 32 64; do echo "redblocks=$rb"; PE_REDBLOCKS=$rb timeout -k 10 60 $BIN --json $ARGS | grep -o '"iters_per_s": [0-9.]*' || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $BIN $ARGS > $O/kt.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/p1 -o run -- $BIN $ARGS > $O/p1.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/p2 -o run -- $BIN $ARGS > $O/p2.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU -d $O/p3 -o run -- $BIN $ARGS > $O/p3.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum -d $O/p4 -o run -- $BIN $ARGS > $O/p4.log 2>&1
echo EXIT $?

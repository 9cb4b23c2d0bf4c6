# Single-sweep kernel tuning sweep (rows per item × register cap) at 8192²,
# then PMC counters of the default configuration.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/fsweep; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
( for occ in 0 4; do for ti in 8 12 16 24 32; do
    echo "occ=$occ ti=$ti"; PE_SOCC=$occ PE_TI=$ti timeout -k 10 100 $BIN --json --quiet --max-iter 600 --no-tol 8192 8192 || exit 1
  done; done ) > $O/sweep.txt 2>&1 || { echo sweep failed; tail $O/sweep.txt; exit 1; }
grep -E "occ=|iters_per_s" $O/sweep.txt | paste - - | sed 's/"timers.*iters_per_s"/ ips/' | cut -c1-200
cd /tmp && export TMPDIR=/tmp
ARGS="--max-iter 60 --no-tol 8192 8192"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $BIN $ARGS > $O/kt.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES -d $O/p1 -o run -- $BIN $ARGS > $O/p1.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/p2 -o run -- $BIN $ARGS > $O/p2.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/p3 -o run -- $BIN $ARGS > $O/p3.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR -d $O/p4 -o run -- $BIN $ARGS > $O/p4.log 2>&1
echo EXIT $?

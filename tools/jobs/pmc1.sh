set -o pipefail
cd /tmp && export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc1
mkdir -p $OUT
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
ARGS="--max-iter 60 --no-tol --variant ${VARIANT:-0} 8192 8192"
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES -d $OUT/p1 -o run -- $BIN $ARGS > $OUT/p1.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/p2 -o run -- $BIN $ARGS > $OUT/p2.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/p3 -o run -- $BIN $ARGS > $OUT/p3.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR -d $OUT/p4 -o run -- $BIN $ARGS > $OUT/p4.log 2>&1
echo EXIT $?

# HBM traffic of the current single-sweep kernels at 8192² (FETCH_SIZE / WRITE_SIZE per dispatch,
# each counter set in its own rocprofv3 pass, --kernel-trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/hbm; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
ARGS="--quiet --max-iter 300 --no-tol 8192 8192"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/p1 -o run -- $BIN $ARGS > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/p2 -o run -- $BIN $ARGS > $O/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/p3 -o run -- $BIN $ARGS > $O/p3.log 2>&1
echo EXIT $?

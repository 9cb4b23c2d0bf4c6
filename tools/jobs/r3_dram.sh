# DRAM requests of the two-step sweep at 8192^2 (read = TCC_EA0_RDREQ x 128 B? see r2 note; write = WRREQ x 64 B)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/dram3; mkdir -p $O
BIN=$R/bin/pe_hip
cd /tmp && export TMPDIR=/tmp
for ti in ${TIS:-40}; do
PE_TI=$ti timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/p_$ti -o run -- $BIN --quiet --max-iter 300 --no-tol ${GRID:-8192 8192} > $O/p_$ti.log 2>&1 || exit 1
done
cd $R
for ti in ${TIS:-40}; do
  db=$(ls $O/p_$ti/run_results.db $O/p_$ti/*/run_results.db 2>/dev/null | tail -1)
  echo "== ti $ti"; python3 tools/pmc_by_dispatch.py $db --kernel kS2 --by-name || exit 1
done
echo EXIT 0

# Counters of the three-step sweep kS3 at ${GRID:-8192 8192} (pe_hip, 300 iterations, tol off), one set per pass
# -> profiles/r3_three_profile.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/three3; mkdir -p $O
BIN=$R/bin/pe_hip
ARGS="--quiet --max-iter 300 --no-tol ${GRID:-8192 8192}"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM" ${EXTRA_SETS}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $O/p$i -o run -- $BIN $ARGS > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
cd $R
for p in $(seq 1 $i); do
  db=$(ls $O/p$p/run_results.db $O/p$p/*/run_results.db 2>/dev/null | tail -1)
  echo "== p$p ($db)"; python3 tools/pmc_by_dispatch.py $db --kernel ${KERN:-kS3} --by-name || exit 1
done
echo EXIT 0

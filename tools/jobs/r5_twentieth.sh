# Round 5, twentieth GPU call: is the sweep clock-bound?  In-kernel shader
# clock (Δ s_memtime / Δ s_memrealtime per wave, stamped build) at 8192^2 and
# the 8-rank slab, and the SQ issue picture of the production kS3 at 8192^2
# (pe_hip, 300 iterations): wave cycles split into active / waiting /
# issue-stalled, VALU and LDS activity, GRBM_GUI_ACTIVE (effective clock).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5twentieth; mkdir -p $O
cd $R
PROBE_CFG=1:device,8:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -h -E "^P=|shader clock|busy fraction" $O/stamps.txt
BIN=$R/bin/pe_hip
ARGS="--quiet --max-iter 300 --no-tol 8192 8192"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d $O/p$i -o run -- $BIN $ARGS > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
cd $R
for p in $(seq 1 $i); do
  db=$(ls $O/p$p/run_results.db $O/p$p/*/run_results.db 2>/dev/null | tail -1)
  echo "== p$p"; python3 tools/pmc_by_dispatch.py $db --kernel kS3 --by-name || exit 1
done
echo EXIT 0

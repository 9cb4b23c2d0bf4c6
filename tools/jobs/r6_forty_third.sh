# Round 6, forty-third GPU call: DRAM bytes and the SQ issue picture of the
# production kS3 at 8192² at the final HEAD (pe_hip, 300 iterations, no stop
# test), one counter pass per run.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fortythird; mkdir -p $O
BIN=$R/bin/pe_hip
ARGS="--quiet --max-iter 300 --no-tol 8192 8192"
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set -d $O/p$i -o run -- $BIN $ARGS > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
cd $R
for p in $(seq 1 $i); do
  db=$(ls $O/p$p/run_results.db $O/p$p/*/run_results.db 2>/dev/null | tail -1)
  echo "== p$p"; python3 tools/pmc_by_dispatch.py $db --kernel kS3 --by-name || exit 1
done
echo EXIT 0

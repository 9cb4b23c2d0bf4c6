# DRAM-side request counters (TCC_EA0_RDREQ x 128 B, TCC_EA0_WRREQ x 64 B) of the
# three-step sweep kS3 at 8192^2 (pe_hip, 300 iterations, tol off) under the
# round-4 layouts (LPT, filling, equal-cost) on 8192^2 and the 8-rank
# slab block (GRID=1024 8191) -> profiles/r4_dram.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${DRAM_OUT:-r4dram}; mkdir -p $O
BIN=$R/bin/pe_hip
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in ${CFGS:-"PE_LAYOUT=lpt" "PE_LAYOUT=fill" "PE_LAYOUT=equal"}; do
  i=$((i+1))
  echo "$cfg" > $O/c$i.cfg
  env $cfg timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/p$i -o run -- $BIN --quiet --max-iter 300 --no-tol ${GRID:-8192 8192} > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
cd $R
for p in $(seq 1 $i); do
  db=$(ls $O/p$p/run_results.db $O/p$p/*/run_results.db 2>/dev/null | tail -1)
  echo "== $(cat $O/c$p.cfg)"; python3 tools/pmc_by_dispatch.py $db --kernel kS3 --by-name || exit 1
done
echo EXIT 0

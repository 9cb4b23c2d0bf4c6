# Profile of the headline at the round's final layout (8192^2, static 24-row LPT items):
# rocprofv3 --kernel-trace --stats of bench.py, then HBM counters of the two sweep
# variants (one counter set per pass, --kernel-trace only) -> profiles/r2_head_profile.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/head; mkdir -p $O
BIN=$R/bin/pe_hip
ARGS="--quiet --max-iter 300 --no-tol 8192 8192"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/bench.py --steps 400 --warmup 20 --no-solve > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/p1 -o run -- $BIN $ARGS > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/p2 -o run -- $BIN $ARGS > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/p3 -o run -- $BIN $ARGS > $O/p3.log 2>&1 || exit 1
cd $R
db=$(ls $O/kt/run_results.db $O/kt/*/run_results.db 2>/dev/null | tail -1)
echo "== bench.py --steps 400 kernel trace ($db)"; python3 tools/rocpd_summary.py $db --timeline 6 || exit 1
grep '^{' $O/kt.log || true
for p in p1 p2 p3; do
  db=$(ls $O/$p/run_results.db $O/$p/*/run_results.db 2>/dev/null | tail -1)
  echo "== $p ($db)"; python3 tools/pmc_by_dispatch.py $db --kernel kS --by-name || exit 1
done
echo EXIT 0

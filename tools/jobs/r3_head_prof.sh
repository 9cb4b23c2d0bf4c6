# Profile of the headline with the two-step sweep (8192^2): rocprofv3 kernel trace of bench.py,
# then DRAM counters of kS2 (one counter set per pass) -> profiles/r3_head_profile.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/head3; mkdir -p $O
BIN=$R/bin/pe_hip
ARGS="--quiet --max-iter 300 --no-tol 8192 8192"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/bench.py --steps 400 --warmup 20 --no-solve > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/p1 -o run -- $BIN $ARGS > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/p2 -o run -- $BIN $ARGS > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES -d $O/p3 -o run -- $BIN $ARGS > $O/p3.log 2>&1 || exit 1
cd $R
db=$(ls $O/kt/run_results.db $O/kt/*/run_results.db 2>/dev/null | tail -1)
echo "== bench.py --steps 400 kernel trace ($db)"; python3 tools/rocpd_summary.py $db --timeline 6 || exit 1
grep '^{' $O/kt.log || true
for p in p1 p2 p3; do
  db=$(ls $O/$p/run_results.db $O/$p/*/run_results.db 2>/dev/null | tail -1)
  echo "== $p ($db)"; python3 tools/pmc_by_dispatch.py $db --kernel kS2 --by-name || exit 1
done
echo EXIT 0

# Round 2: rocprofv3 kernel traces (durations + dispatch gaps) of the three device paths:
# resident (800x1200), tuned static streaming (2400x3200), dynamic streaming (8192^2).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r2prof; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
cd /tmp && export TMPDIR=/tmp
for g in "800 1200 1024" "2400 3200 600" "8192 8192 200"; do
  set -- $g
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$1x$2 -o run -- $BIN --quiet --max-iter $3 --no-tol $1 $2 > $O/kt_$1x$2.log 2>&1 || { tail -20 $O/kt_$1x$2.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for n in 800x1200 2400x3200 8192x8192; do
  db=$(ls $O/kt_$n/*/run_results.db $O/kt_$n/run_results.db 2>/dev/null | head -1)
  echo "== $n ($db)"; python3 tools/rocpd_summary.py $db --timeline 8 || true
  st=$(ls $O/kt_$n/*/run_kernel_stats.csv $O/kt_$n/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$st" ] && { echo "-- kernel stats csv"; head -12 $st; }
done
echo EXIT 0

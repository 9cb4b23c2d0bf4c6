# Round 2: where do small / medium grids spend their per-iteration time?
# Full solves + kernel traces (durations and inter-dispatch gaps) + in-kernel stamps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/small2; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
for g in "800 1200" "2400 3200"; do
  timeout -k 10 60 $BIN --json $g || exit 1
done
cd /tmp && export TMPDIR=/tmp
for g in "800 1200" "2400 3200"; do
  n=${g/ /x}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o run -- $BIN --quiet --max-iter 600 --no-tol $g > $O/kt_$n.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for n in 800x1200 2400x3200; do
  db=$(ls $O/kt_$n/*/run_results.db $O/kt_$n/run_results.db 2>/dev/null | head -1)
  echo "== $n $db"; python3 tools/rocpd_summary.py $db --timeline 12 || true
done
PROBE_GRID=800x1200 PROBE_CFG=1:aspect timeout -k 10 120 python3 -u tools/stamp_probe.py > $O/stamp_800.txt 2>&1 || exit 1
cat $O/stamp_800.txt
PROBE_GRID=2400x3200 PROBE_CFG=1:aspect timeout -k 10 120 python3 -u tools/stamp_probe.py > $O/stamp_2400.txt 2>&1 || exit 1
cat $O/stamp_2400.txt
echo EXIT 0

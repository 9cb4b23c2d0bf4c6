# Round 2: per-row-step timeline of the first item of every wave (PE_STAMPS build).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/steps; mkdir -p $O
for g in 800x1200 2400x3200 8192x8192; do
  PROBE_GRID=$g PROBE_CFG=1:aspect timeout -k 10 120 python3 -u tools/stamp_probe.py > $O/stamp_$g.txt 2>&1 || exit 1
  cat $O/stamp_$g.txt | grep -v "late item"
done
echo EXIT 0

# Round 2: LDS-resident single sweep — correctness (golden counts, resident vs
# streaming) and per-iteration time on the small grids.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/resident; mkdir -p $O
for g in "40 40" "400 600" "800 1200" "1024 1024" "1200 1600"; do
  for r in 1 0; do
    PE_RESIDENT=$r timeout -k 10 60 bin/pe_hip --json $g > $O/g_${g/ /x}_$r.json 2> $O/g_${g/ /x}_$r.err || { cat $O/g_${g/ /x}_$r.err; exit 1; }
    echo "PE_RESIDENT=$r $(tail -1 $O/g_${g/ /x}_$r.json)"
  done
done
echo EXIT 0

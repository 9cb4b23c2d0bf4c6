# Round 6, twenty-sixth GPU call: the filling layout's pass loop oscillates on
# blocks of about one item per wave (1791 / 88 cuts, r6_twenty_fifth); the
# overlap timed at its three heights with the last pass (mode 0), the pass of
# the lowest estimated makespan (1) and no cuts (2): 8-rank slab and 4x2.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twentysixth; mkdir -p $O
cd $R
for spec in rows 4x2; do
  for m in 0 1 2; do
    PE_FILL_MODE=$m PROBE_SPEC=$spec PROBE_REPS=2 timeout -k 10 200 python -u tools/overlap_trace_probe.py > $O/ov_${spec}_$m.txt 2>&1 || { tail -20 $O/ov_${spec}_$m.txt; exit 1; }
    echo "== $spec mode $m"; grep "^rep" $O/ov_${spec}_$m.txt | sed 's/tuning \[.*\]; halo/halo/' | cut -c1-330
  done
done
echo EXIT 0

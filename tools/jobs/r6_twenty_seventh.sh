# Round 6, twenty-seventh GPU call: where a fresh process's construction goes
# on the small / mid BASELINE grids (T_solver includes it: 25 % at 2048²) —
# PE_CTOR_TRACE=3 (phases + layout laps), bin/pe_hip --json.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twentyseventh; mkdir -p $O
cd $R
for g in "2048 2048" "1600 2400" "2400 3200" "4096 4096"; do
  PE_CTOR_TRACE=3 timeout -k 10 120 bin/pe_hip --json $g > $O/grid_${g/ /x}.json 2> $O/grid_${g/ /x}.err || { tail -5 $O/grid_${g/ /x}.err; exit 1; }
  echo "== $g"; grep -E "ctor|layout (lpt|equal|fill|list)" $O/grid_${g/ /x}.err | head -80
done
echo EXIT 0

# Round 5, twenty-first GPU call: where the construction time of the small
# BASELINE grids goes (PE_CTOR_TRACE=1: allocation, tables, layout, tuning),
# T_solver vs T_iterate at 2048^2, 1600x2400, 2400x3200, 4096^2 (pe_hip, 2 runs each).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5twentyfirst; mkdir -p $O
cd $R
for g in "2048 2048" "1600 2400" "2400 3200" "4096 4096"; do
  for rep in 1 2; do
    PE_CTOR_TRACE=1 timeout -k 10 60 bin/pe_hip --json $g > $O/run.json 2> $O/ctor.txt || { tail -5 $O/ctor.txt; exit 1; }
    echo "== $g rep $rep"; grep "\[pe\] ctor" $O/ctor.txt | head -40
    python3 -c "
import json
d=json.load(open('$O/run.json')); t=d.get('timers', d)
print('iters', d.get('iters'), {k: t[k] for k in t if isinstance(t[k], (int, float)) and k in ('solver','setup','iterate','check','gpu','t_solver','t_setup','t_iterate')})" 2>/dev/null || tail -3 $O/run.json
  done
done
echo EXIT 0

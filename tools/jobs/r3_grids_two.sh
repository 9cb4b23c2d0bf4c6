# Round 3: published / BASELINE grids, default algorithm vs the two-step sweep (fresh processes).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3grids; mkdir -p $O
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  for algo in auto two-step; do
    f=$O/g_${g/ /x}_$algo.json
    timeout -k 10 120 bin/pe_hip --json --algo $algo $g > $f 2>&1 || { cat $f; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$g', '$algo', d['algo'], d['iters'], 'T_solver %.4f' % d['t_solver'], 'iter/s %.1f' % (d['iters']/d['t_iterate']), 'L2 %.4e' % d['l2_err'])" 2>/dev/null || tail -2 $f
  done
done
echo EXIT 0

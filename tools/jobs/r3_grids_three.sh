# Round 3: published / BASELINE grids, default algorithm (three-step where it applies) vs the
# two-step sweep (fresh processes); then smoke and the driver-shaped bench runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3grids3; mkdir -p $O
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  for algo in auto two-step; do
    f=$O/g_${g/ /x}_$algo.json
    timeout -k 10 120 bin/pe_hip --json --algo $algo $g > $f 2>&1 || { cat $f; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$g', '$algo', d['algo'], d['iters'], 'T_solver %.4f' % d['t_solver'], 'iter/s %.1f' % (d['iters']/d['t_iterate']), 'L2 %.4e' % d['l2_err'])" 2>/dev/null || tail -2 $f
  done
done
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || { tail $O/bench2000.err; exit 1; }
cat $O/bench2000.json
echo EXIT 0

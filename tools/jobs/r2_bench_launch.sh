# bench.py timed steps: graph replay vs eager launches, same box, alternating (fresh process each).
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
 for l in graph eager; do
  for st in 20 400; do
   timeout -k 10 120 python -u bench.py --steps $st --warmup 5 --no-solve --launch $l 2>/dev/null | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); print('$l steps $st', round(d['value'],1), 'ms/step %.4f' % d['ms_per_step'], d['config']['placement']['candidates_ms_per_sweep'])" || exit 1
  done
 done
done

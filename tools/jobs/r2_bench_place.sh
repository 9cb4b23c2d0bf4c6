# bench.py with the placement search keeping the best of all tries (fresh process each).
cd $GRAFT_REPO_ROOT
for r in 1 2 3 4; do
  timeout -k 10 120 python -u bench.py --steps 400 --warmup 5 --no-solve 2>/dev/null | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); c=d['config']; print(round(d['value'],1), 'ms/step %.4f' % d['ms_per_step'], c['placement'], 'construct %.3f' % c['construct_s'])" || exit 1
done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 2>/dev/null | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); c=d['config']; print('steps 20 + solve:', round(d['value'],1), c['placement'], 't_solver %.3f setup %.3f' % (d['t_solver_s'], d['t_setup_s']), d['iters_converged'])" || exit 1

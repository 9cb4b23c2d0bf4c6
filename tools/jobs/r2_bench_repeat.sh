# Headline bench in N fresh processes (placement search outcome per process) -> profiles/r2_bench_repeat.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in $(seq ${REPEAT:-4}); do
  timeout -k 10 120 python3 -u bench.py --steps ${STEPS:-20} --warmup 5 > gpurun_out/rep_$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/rep_$i.json')); p=d['config']['placement']; print('%.1f it/s' % d['value'], 'T_solver %.3f' % d['t_solver_s'], 'iters', d['iters_converged'], 'placement', p['candidates_ms_per_sweep'], 'chosen', p['chosen'], 'search %.3f s' % p['search_s'])" || exit 1
done
echo EXIT 0

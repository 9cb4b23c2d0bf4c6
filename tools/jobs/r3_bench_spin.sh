# bench.py --steps 20 --warmup 5 in 4 fresh processes after the event-wait spin change
set -o pipefail
cd $GRAFT_REPO_ROOT; O=$GRAFT_REPO_ROOT/gpurun_out/bspin; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 > $O/b$i.json 2> $O/b$i.err || { tail $O/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$i.json')); print('bench20 run $i', round(d['value'],1), 'it/s', round(d['ms_per_step'],4), 'ms/step', d['config']['launch'], 'job', d['config']['placement']['job_ms_per_sweep'], 'solve it/s', round(d['solve_iters_per_s'],1), 't_solver', d['t_solver_s'])"
done
echo EXIT 0

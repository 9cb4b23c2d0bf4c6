# bench.py after the clock warm-up (--warmup-s 0.25 default) and the 4.4 TB/s
# placement stop: three driver-shaped 20-step runs, one 2000-step run, fresh
# processes -> profiles/r4_bench_warm.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/bw_$i.json 2> $O/bw_$i.err || { tail $O/bw_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bw_$i.json')); print('bench20 run $i', round(d['value'],1), round(d['ms_per_step'],4), 'clock warm-up', d['clock_warmup_steps'], d['config']['placement'])"
done
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bw_long.json 2> $O/bw_long.err || { tail $O/bw_long.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bw_long.json')); print('bench2000', round(d['value'],1), round(d['ms_per_step'],4), d['config']['placement'])"
timeout -k 10 180 python -u bench.py > $O/bw_default.json 2> $O/bw_default.err || { tail $O/bw_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bw_default.json')); print('bench default', d['steps'], d['warmup'], round(d['value'],1), round(d['ms_per_step'],4), 'T_solver', d.get('t_solver_s'), 'iters', d.get('iters_converged'))"
echo EXIT 0

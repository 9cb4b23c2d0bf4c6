# Round-4 final check at HEAD: three-step / residual / layout GPU tests,
# published / BASELINE grids in fresh processes, bench 20 (x2) / 2000 steps,
# smoke() -> profiles/r4_final.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4final; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --tb=short --timeout 240 --timeout-method thread tests/test_three_step.py tests/test_residual.py tests/test_layout.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  f=$O/g_${g/ /x}.json
  timeout -k 10 120 bin/pe_hip --json --quiet $g > $f 2>&1 || { cat $f; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$g', d['algo'], d['iters'], 'T_solver %.4f' % d['t_solver'], 'construct %.4f' % d['t_construct'],
      'iterate %.4f' % d['t_iterate'], 'gpu %.4f copy %.4f' % (d['t_gpu'], d['t_copy']), 'L2 %.4e' % d['l2_err'], 'res_gap %.2e' % d['res_gap'], 'restarts %d' % d['restarts'])"
done
for i in 1 2; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench20_$i.json 2> $O/bench20_$i.err || { tail $O/bench20_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench20_$i.json')); print('bench20 run $i', round(d['value'],1), round(d['ms_per_step'],4), 'T_solver', d.get('t_solver_s'), 'random', d.get('random_init',{}).get('iters'), d['config']['placement']['job_ms_per_sweep'])"
done
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || { tail $O/bench2000.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench2000.json')); print('bench2000', round(d['value'],1), round(d['ms_per_step'],4), d['config']['placement']['job_ms_per_sweep'])"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
echo EXIT 0

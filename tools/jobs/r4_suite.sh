# Round-4 validation at HEAD: the whole GPU suite, the driver's smoke(),
# published / BASELINE grids in fresh processes (T_solver with the Table-2
# breakdown; 400x600 first, on a fresh box), bench 20 / 2000 steps
# -> profiles/r4_suite.txt, profiles/r4_grids.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4suite; mkdir -p $O
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  f=$O/g_${g/ /x}.json
  PE_CTOR_TRACE=1 timeout -k 10 120 bin/pe_hip --json --quiet $g > $f 2>&1 || { cat $f; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$g', d['algo'], d['iters'], 'T_solver %.4f' % d['t_solver'], 'construct %.4f' % d['t_construct'],
      'iterate %.4f' % d['t_iterate'], 'gpu %.4f copy %.4f halo %.4f reduce %.4f dot %.4f' % (d['t_gpu'], d['t_copy'], d['t_halo'], d['t_reduce'], d['t_dot']),
      'L2 %.4e' % d['l2_err'], 'res_gap %.2e' % d['res_gap'], 'restarts %d' % d['restarts'])" || tail -2 $f
done
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench20.json')); print('bench20', round(d['value'],1), round(d['ms_per_step'],4), 'T_solver', d.get('t_solver_s'), 'random', d.get('random_init',{}).get('iters'))"
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || { tail $O/bench2000.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench2000.json')); print('bench2000', round(d['value'],1), round(d['ms_per_step'],4))"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 240 --timeout-method thread > $O/suite.txt 2>&1 || { tail -30 $O/suite.txt; exit 1; }
tail -3 $O/suite.txt
echo EXIT 0

# Round 6, tenth GPU call: smoke, the whole GPU suite at HEAD, then a
# same-box A/B of the 1-GPU bench (HEAD vs round 5, 4 alternating pairs).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6tenth; mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for i in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/head_$i.txt 2>&1 || { tail -20 $O/head_$i.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/head_$i.txt').read().strip().splitlines()[-1]);print('HEAD',round(d['value'],1),d['config']['placement']['candidates_ms_per_sweep'][d['config']['placement']['chosen']],round(d['t_solver_s'],4))"
  timeout -k 10 200 python -u .r5ref/bench.py --steps 20 --warmup 5 --no-random-solve > $O/r5_$i.txt 2>&1 || { tail -20 $O/r5_$i.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/r5_$i.txt').read().strip().splitlines()[-1]);print('R5  ',round(d['value'],1),d['config']['placement']['candidates_ms_per_sweep'][d['config']['placement']['chosen']],round(d['t_solver_s'],4))"
done
echo EXIT 0

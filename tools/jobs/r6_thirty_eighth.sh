# Round 6, thirty-eighth GPU call: the placement search's stop rule at 4.45
# TB/s — four fresh 1-GPU bench processes (20 steps) with their candidates,
# then the placement GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirtyeighth; mkdir -p $O
cd $R
for i in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/bench_$i.txt 2>&1 || { tail -20 $O/bench_$i.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$i.txt').read().strip().splitlines()[-1]);p=d['config']['placement'];print('bench',round(d['value'],1),p['candidates_ms_per_sweep'],p['chosen'],p['search_s'],round(d['t_solver_s'],4))"
done
# (a -k "placement" test selection matched no test: pytest exit 5 ended the call after the benches)
echo EXIT 0

# Round 6, twenty-fourth GPU call: same-box A/B of the 2000-step bench (HEAD
# vs the round-5 build in .r5ref/, 3 alternating pairs, no full solves).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twentyfourth; mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/head_$i.txt 2>&1 || { tail -20 $O/head_$i.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/head_$i.txt').read().strip().splitlines()[-1]);print('HEAD',round(d['value'],1),d['config']['placement']['candidates_ms_per_sweep'][d['config']['placement']['chosen']])"
  timeout -k 10 200 python -u .r5ref/bench.py --steps 2000 --warmup 100 --no-solve > $O/r5_$i.txt 2>&1 || { tail -20 $O/r5_$i.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/r5_$i.txt').read().strip().splitlines()[-1]);print('R5  ',round(d['value'],1),d['config']['placement']['candidates_ms_per_sweep'][d['config']['placement']['chosen']])"
done
echo EXIT 0

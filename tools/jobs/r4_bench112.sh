# bench.py with 112-row items at 8192^2 (aligned strips): three driver-shaped
# 20-step runs and one 2000-step run in fresh processes, with each run's
# placement candidates; 16384^2 golden + residual gap (256-row items) -> profiles/r4_bench112.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/b112_$i.json 2> $O/b112_$i.err || { tail $O/b112_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b112_$i.json')); print('bench20 run $i', round(d['value'],1), round(d['ms_per_step'],4), d['config']['rows_per_item'], d['config']['placement'])"
done
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/b112_long.json 2> $O/b112_long.err || { tail $O/b112_long.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b112_long.json')); print('bench2000', round(d['value'],1), round(d['ms_per_step'],4), d['config']['placement'])"
timeout -k 10 120 bin/pe_hip --json --quiet 16384 16384 > $O/b112_16k.json 2>&1 || { cat $O/b112_16k.json; exit 1; }
grep "^{" $O/b112_16k.json
echo EXIT 0

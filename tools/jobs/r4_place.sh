# Placement landscape of the three-step sweep at 8192^2 (112-row items): every
# candidate of a long search (24 tries, no early stop, 85 % of free memory,
# 5 s cap), two fresh processes -> profiles/r4_place.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
for i in 1 2; do
  PE_PLACEMENT_TRIES=24 PE_PLACEMENT_FAST_TBS=100 PE_PLACEMENT_MAX_S=5 PE_PLACEMENT_MEM_FRAC=0.85 timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/pl_$i.json 2> $O/pl_$i.err || { tail $O/pl_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/pl_$i.json')); print('run $i', round(d['value'],1), round(d['ms_per_step'],4), d['config']['placement'])"
done
echo EXIT 0

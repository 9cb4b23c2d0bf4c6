# Round 5, eighteenth GPU call: neighbouring strips in one L2 without the
# whole-range XCD map — runs of g consecutive lists' workgroups on one XCD
# (PE_XCD_GROUP = 1 default, 2, 4, 8): 8192^2 it/s and DRAM request counters.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5eighteenth; mkdir -p $O
cd $R
for rep in 1 2; do
  for g in 1 2 4 8; do
    PE_XCD_GROUP=$g timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/b_${g}_$rep.json 2> $O/b_${g}_$rep.err || { tail -5 $O/b_${g}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${g}_$rep.json').read().strip().splitlines()[-1]); print('group $g', round(d['value'],1), 'iters', d.get('iters_converged'), 't_iterate', d.get('t_iterate_s'))"
  done
done
for g in 2 4; do
  PE_XCD_GROUP=$g PROBE_CFG=8:device,8:4x2 timeout -k 10 120 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/group $g /"
done
DRAM_OUT=r5eighteenth/dram CFGS="PE_XCD_GROUP=1 PE_XCD_GROUP=2 PE_XCD_GROUP=4" timeout -k 10 600 bash tools/jobs/r4_dram.sh | sed -n '/^==/,$p'
echo EXIT 0

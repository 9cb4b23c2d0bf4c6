# Round 5, fourteenth GPU call: the SIMD's two waves taking turns at issue
# priority (PE_PRIO = log2 of the turn in 10 ns ticks): stamped timelines
# (per-workgroup speed, SIMD with one wave left) and benches / probes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fourteenth; mkdir -p $O
cd $R
PROBE_ENV="PE_PRIO=0;PE_PRIO=10" PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -h -E "^P=|one wave left|SIMD exit|tail \(|busy fraction|by workgroup decile" $O/stamps.txt
for y in 0 8 10 12 0; do
  PE_PRIO=$y timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/b_$y.json 2> $O/b_$y.err || exit 1
  PE_PRIO=$y timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --grid 2048 2048 > $O/b2048_$y.json 2> $O/b2048_$y.err || exit 1
  PE_PRIO=$y PROBE_CFG=8:device,8:4x2,4:device timeout -k 10 240 python -u tools/block_probe.py > $O/probe_$y.txt 2>&1 || exit 1
  python3 -c "
import json
for n in ('b_$y','b2048_$y'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); print('prio $y', n, round(d['value'],1), 'iters', d.get('iters_converged'), 't_iterate', d.get('t_iterate_s'), d['config']['item_order'], d['config']['rows_per_item'])"
  grep -h "us/iter" $O/probe_$y.txt | sed "s/^/prio $y /"
done
echo EXIT 0

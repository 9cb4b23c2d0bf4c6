# Round 5, fifteenth GPU call: default SIMD priority turns below 6e6 nodes —
# A/B against PE_PRIO=0 on the small grids (1-GPU full solves and 2-rank blocks).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fifteenth; mkdir -p $O
cd $R
for g in "2048 2048" "1600 2400" "2400 3200"; do
  n=$(echo $g | tr ' ' x)
  for v in def 0 def 0; do
    if [ $v = def ]; then E=""; else E="PE_PRIO=0"; fi
    env $E timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --grid $g --no-random-solve > $O/b_${n}_$v.json 2> $O/b_${n}_$v.err || exit 1
    python3 -c "
import json
d=json.loads(open('$O/b_${n}_$v.json').read().strip().splitlines()[-1]); print('$n', '$v', round(d['value'],1), 'iters', d.get('iters_converged'), 't_solver', round(d.get('t_solver_s'),5), 't_iterate', round(d.get('t_iterate_s'),5), d['config']['item_order'], d['config']['rows_per_item'], d['config']['resident'])"
  done
done
for v in "" "PE_PRIO=0"; do
  PROBE_ENV="$v" PROBE_GRID=2048x2048 PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py 2>&1 | grep "us/iter"
  PROBE_ENV="$v" PROBE_GRID=1600x2400 PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py 2>&1 | grep "us/iter"
  PROBE_ENV="$v" PROBE_GRID=4096x4096 PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py 2>&1 | grep "us/iter"
done
echo EXIT 0

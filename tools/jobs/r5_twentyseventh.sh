# Round 5, twenty-seventh GPU call: rows per item at 8192^2 after the round-5
# epilogue / prologue changes (PE_TI, LPT layout; round 4: 112 and 132 best).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5twentyseventh; mkdir -p $O
cd $R
for rep in 1 2; do
  for ti in 112 96 104 120 132 144; do
    PE_TI=$ti timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/b_${ti}_$rep.json 2> $O/b_${ti}_$rep.err || { tail -5 $O/b_${ti}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${ti}_$rep.json').read().strip().splitlines()[-1]); print('ti $ti', round(d['value'],1), 'iters', d.get('iters_converged'), 't_iterate', d.get('t_iterate_s'), d['config']['rows_per_item'], d['config']['ranks'][0]['pci_bus_id'])"
  done
done
echo EXIT 0

# Round 5, seventeenth GPU call: where the 8192^2 sweep's read excess goes —
# one tall segment per wave (PE_SEGMENTS=1: no refill rows between a wave's
# items) and the XCD-contiguous list map (PE_XCD_MAP=1: neighbouring strips'
# shared halo lines in one L2) against the default LPT items: it/s and DRAM
# request counters (TCC_EA0_RDREQ x 128 B, TCC_EA0_WRREQ x 64 B).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5seventeenth; mkdir -p $O
cd $R
for rep in 1 2; do
  for cfg in PE_LAYOUT=lpt PE_SEGMENTS=1 PE_XCD_MAP=1; do
    env $cfg timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/b_${cfg}_$rep.json 2> $O/b_${cfg}_$rep.err || { tail -5 $O/b_${cfg}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${cfg}_$rep.json').read().strip().splitlines()[-1]); print('$cfg', round(d['value'],1), 'iters', d.get('iters_converged'), 't_iterate', d.get('t_iterate_s'), d['config']['item_order'], d['config']['rows_per_item'])"
  done
done
for cfg in PE_LAYOUT=lpt PE_SEGMENTS=1 PE_XCD_MAP=1; do
  env $cfg PROBE_CFG=8:device timeout -k 10 120 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/$cfg /"
done
DRAM_OUT=r5seventeenth/dram CFGS="PE_LAYOUT=lpt PE_SEGMENTS=1 PE_XCD_MAP=1" timeout -k 10 600 bash tools/jobs/r4_dram.sh | sed -n '/^==/,$p'
echo EXIT 0

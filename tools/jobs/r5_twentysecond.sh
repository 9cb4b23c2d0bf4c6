# Round 5, twenty-second GPU call: L2 prefetch of the steady row groups
# (PE_PF = rows beyond the register prefetch, LDS-DMA into a scratch slot):
# 8192^2 it/s and the stamped wave wait picture at PE_PF 0 / 2 / 4 / 8.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5twentysecond; mkdir -p $O
cd $R
for rep in 1 2; do
  for pf in 0 2 4 8; do
    PE_PF=$pf timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/b_${pf}_$rep.json 2> $O/b_${pf}_$rep.err || { tail -5 $O/b_${pf}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${pf}_$rep.json').read().strip().splitlines()[-1]); print('pf $pf', round(d['value'],1), 'iters', d.get('iters_converged'), 't_iterate', d.get('t_iterate_s'), d['config']['ranks'][0]['pci_bus_id'])"
  done
done
for pf in 0 4; do
  PE_PF=$pf PROBE_CFG=8:device,8:4x2 timeout -k 10 120 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/pf $pf /"
done
echo EXIT 0

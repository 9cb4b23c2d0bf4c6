# Round 5, eleventh GPU call: (1) the new sweep epilogue (n-major partials,
# DPP wave sums, pending records from kernel entry) in the stamped timeline;
# (2) wave-age capacity rho (PE_YOUNG) for the fill / LPT layouts: per-rank
# probes, 8192^2 and 2048^2 benches at rho 1.0 / 1.1 / 1.2 / 1.3.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5eleventh; mkdir -p $O
cd $R
PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -h -E "^P=|last block|last wave exit|busy fraction|by workgroup decile" $O/stamps.txt
PE_YOUNG=1.2 PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps_y12.txt 2>&1 || { tail -20 $O/stamps_y12.txt; exit 1; }
grep -h -E "^P=|last wave exit|busy fraction|by workgroup decile|tail \(" $O/stamps_y12.txt
for y in 1.0 1.1 1.2 1.3; do
  PE_YOUNG=$y timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/b_$y.json 2> $O/b_$y.err || exit 1
  PE_YOUNG=$y timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --grid 2048 2048 > $O/b2048_$y.json 2> $O/b2048_$y.err || exit 1
  PE_YOUNG=$y PROBE_CFG=8:device,8:4x2,4:device timeout -k 10 240 python -u tools/block_probe.py > $O/probe_$y.txt 2>&1 || exit 1
  python3 -c "
import json
for n in ('b_$y','b2048_$y'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); print('rho $y', n, round(d['value'],1), 'iters', d.get('iters_converged'), 't_iterate', d.get('t_iterate_s'), d['config']['item_order'], d['config']['rows_per_item'])"
  grep -h "us/iter" $O/probe_$y.txt | sed "s/^/rho $y /"
done
echo EXIT 0

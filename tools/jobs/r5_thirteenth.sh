# Round 5, thirteenth GPU call: where the waves run (HW_ID / XCC_ID stamps) —
# per-SIMD and per-CU exits: is the sweep's tail whole SIMDs idle, or SIMDs
# down to one wave?  8-rank slab, 2048^2, 8192^2; then the HEAD benches.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirteenth; mkdir -p $O
cd $R
PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
PROBE_GRID=2048x2048 PROBE_CFG=1:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps2048.txt 2>&1 || { tail -20 $O/stamps2048.txt; exit 1; }
grep -h -E "^P=|placement|exit \(its|one wave left|tail \(|busy fraction|busy waves" $O/stamps.txt $O/stamps2048.txt
for i in 1 2; do timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/b$i.json 2> $O/b$i.err || exit 1; done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --grid 2048 2048 > $O/b2048.json 2> $O/b2048.err || exit 1
python3 -c "
import json
for n in ('b1','b2','b2048'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); print(n, round(d['value'],1), d.get('iters_converged'), 't_solver', d.get('t_solver_s'), 't_iterate', d.get('t_iterate_s'), d['config']['ranks'][0]['pci_bus_id'])"
PROBE_CFG=8:device,8:4x2,4:device,2:device timeout -k 10 240 python -u tools/block_probe.py > $O/probe.txt 2>&1 || exit 1
grep -h "us/iter" $O/probe.txt
echo EXIT 0

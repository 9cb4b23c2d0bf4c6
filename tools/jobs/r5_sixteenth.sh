# Round 5, sixteenth GPU call: HEAD numbers for docs/PERFORMANCE.md —
# 1-GPU benches (20 and 2000 steps), every per-rank block projection
# (8192^2 2/4/8 and 4x2, 16384^2 2/4/8, 4096^2 and the reference's 2-GPU grids
# on 2 ranks), the 4x2 overlap at 15 / 8 us delays, the stamped slab timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5sixteenth; mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/head_$i.json 2> $O/head_$i.err || { tail -5 $O/head_$i.err; exit 1; }
done
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 5 --no-random-solve > $O/head_2000.json 2> $O/head_2000.err || { tail -5 $O/head_2000.err; exit 1; }
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --grid 2048 2048 > $O/head_2048.json 2> $O/head_2048.err || exit 1
python3 -c "
import json,glob,os
for f in sorted(glob.glob('$O/head_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(os.path.basename(f)[:-5], round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), d.get('iters_converged'), 't_solver', d.get('t_solver_s'), 't_iterate', d.get('t_iterate_s'), d['config']['ranks'][0]['pci_bus_id'])"
PROBE_CFG=2:device,4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe_8192.txt 2>&1 || exit 1
PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_CFG=2:device,4:device,8:device timeout -k 10 240 python -u tools/block_probe.py > $O/probe_16384.txt 2>&1 || exit 1
for g in 4096x4096 1600x2400 2048x2048 2400x3200 800x1200; do
  PROBE_GRID=$g PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe_$g.txt 2>&1 || exit 1
done
for f in $O/probe_*.txt; do echo "== $(basename $f)"; grep -h "us/iter" $f; done
PROBE_CFG=8:4x2 PROBE_GRAPH=0 timeout -k 10 240 python -u tools/overlap_probe.py 15 8 > $O/overlap.txt 2>&1 || exit 1
grep -h "us/iter" $O/overlap.txt
PROBE_CFG=8:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || exit 1
grep -h -E "us/iter|busy fraction|tail \(max|gap after|walk entry|first item start|last wave exit|last block|one wave left" $O/stamps.txt
echo EXIT 0

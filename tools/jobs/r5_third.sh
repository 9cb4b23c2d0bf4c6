# Round 5, third GPU call: heavy (band) pieces spread over CUs (PE_SPREAD),
# bench A/B (spread vs wave-order ties), block probes, overlap probe,
# stamped timelines -> profiles/r5_*.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5third; mkdir -p $O
cd $R
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || exit 1
  PE_SPREAD=0 timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/benchs$i.json 2> $O/benchs$i.err || exit 1
  PE_SPREAD=0 PE_LPT_KIND=0 timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/benchsk$i.json 2> $O/benchsk$i.err || exit 1
done
python3 -c "
import json
for n in ('bench1','benchs1','benchsk1','bench2','benchs2','benchsk2'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); print(n, round(d['value'],1), round(d['ms_per_step'],4), d.get('iters_converged'), d['config']['placement']['job_ms_per_sweep'], d['config']['ranks'][0]['pci_bus_id'])"
PROBE_CFG=2:device,4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe8192.txt 2>&1 || exit 1
PE_SPREAD=0 PROBE_CFG=8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe8192s.txt 2>&1 || exit 1
for g in 1600x2400 2048x2048; do
  PROBE_GRID=$g PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe$g.txt 2>&1 || exit 1
done
grep -h "us/iter" $O/probe*.txt
PROBE_CFG=8:4x2,4:2x2 PROBE_GRAPH=0 timeout -k 10 240 python -u tools/overlap_probe.py 15 8 > $O/overlap.txt 2>&1 || exit 1
grep -h "us/iter" $O/overlap.txt
PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
grep -h "us/iter\|busy fraction\|tail (max\|band items\|kind " $O/stamps.txt
echo EXIT 0

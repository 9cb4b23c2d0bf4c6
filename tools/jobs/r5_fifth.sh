# Round 5, fifth GPU call: same-box A/B of the round-5 layout changes against
# the round-4 build (.r4ref): 8192^2 bench variants, per-rank block probes,
# stamped 8192^2 timeline -> profiles/r5_ab_layout.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fifth; mkdir -p $O
cd $R
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
}
for i in 1 2; do
  (cd .r4ref && timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/r4_$i.json 2> $O/r4_$i.err) || { tail -5 $O/r4_$i.err; exit 1; }
  run def_$i PE_X=1
  run nospread_$i PE_SPREAD=0
  run nopre_$i PE_PRE=0
  run r4lay_$i PE_LPT_KIND=0 PE_SPREAD=0 PE_PRE=0
done
python3 -c "
import json,glob,os
for f in sorted(glob.glob('$O/*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(os.path.basename(f)[:-5], round(d['value'],1), d['config']['placement']['job_ms_per_sweep'], d['config']['ranks'][0]['pci_bus_id'])"
(cd .r4ref && PROBE_CFG=2:device,4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe_r4.txt 2>&1) || exit 1
PROBE_CFG=2:device,4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe_def.txt 2>&1 || exit 1
PE_SPREAD=0 PROBE_CFG=4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe_nospread.txt 2>&1 || exit 1
for g in 1600x2400 2048x2048 2400x3200; do
  (cd .r4ref && PROBE_GRID=$g PROBE_CFG=1:device,2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe_r4_$g.txt 2>&1) || exit 1
  PROBE_GRID=$g PROBE_CFG=1:device,2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe_def_$g.txt 2>&1 || exit 1
done
for f in $O/probe_*.txt; do echo "== $(basename $f)"; grep -h "us/iter" $f; done
PROBE_CFG=1:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || exit 1
grep -h "us/iter\|kind \|busy fraction\|tail (max" $O/stamps.txt
echo EXIT 0

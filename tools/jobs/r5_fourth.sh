# Round 5, fourth GPU call: is the 8192^2 slowdown the kernel or the box?
# Same box: the round-4 build (.r4ref: HEAD c6b1058's bench.py + extension)
# vs HEAD with PE_DRING=0/1 (band 1/D ring), the round-4 layout
# (PE_LPT_KIND=0 PE_SPREAD=0 PE_PRE=0) and the new defaults
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fourth; mkdir -p $O
cd $R
run() {  # name, env..., then bench args
  local n=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
}
for i in 1 2; do
  (cd .r4ref && timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/r4_$i.json 2> $O/r4_$i.err) || { tail -5 $O/r4_$i.err; exit 1; }
  run oldlay_d1_$i PE_LPT_KIND=0 PE_SPREAD=0 PE_PRE=0 PE_DRING=1
  run oldlay_d0_$i PE_LPT_KIND=0 PE_SPREAD=0 PE_PRE=0 PE_DRING=0
  run new_d1_$i PE_DRING=1
  run new_d0_$i PE_DRING=0
done
python3 -c "
import json,glob,os
for f in sorted(glob.glob('$O/*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(os.path.basename(f)[:-5], round(d['value'],1), d['config']['placement']['job_ms_per_sweep'], d['config']['ranks'][0]['pci_bus_id'])"
PE_LPT_KIND=0 PE_SPREAD=0 PE_PRE=0 PE_DRING=1 PROBE_CFG=1:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps_d1.txt 2>&1 || exit 1
PE_LPT_KIND=0 PE_SPREAD=0 PE_PRE=0 PE_DRING=0 PROBE_CFG=1:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps_d0.txt 2>&1 || exit 1
grep -h "us/iter\|kind \|busy fraction" $O/stamps_d1.txt $O/stamps_d0.txt
echo EXIT 0

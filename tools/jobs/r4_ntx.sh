# kS3 build variants — non-temporal r/p loads (pe_hip_ntx: -DPE_S3_NTX=1),
# 4 prefetched rows (pe_hip_xd4: -DPE_S3_XD=4; pe_hip_xd4ntx both), 2 w rows
# (pe_hip_wd2: -DPE_S3_WD=2) — vs the default build, alternating fresh processes at
# 8192^2 (3000 iterations, tol off; each process runs its own placement
# search), then rows per item around 112 -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
for i in 1 2 3; do
  for b in pe_hip pe_hip_ntx pe_hip_xd4 pe_hip_xd4ntx pe_hip_wd2; do
    timeout -k 10 60 bin/$b --json --quiet --max-iter 3000 --no-tol 8192 8192 > $O/ntx_${b}_${i}.json 2>&1 || { cat $O/ntx_${b}_${i}.json; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('$O/ntx_${b}_${i}.json') if l.startswith('{')][0]
print('$b run $i', 'iterate %.4f s' % d['t_iterate'], 'us/iter %.1f' % (d['t_iterate'] / d['iters'] * 1e6))"
  done
done
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="112 PE_LAYOUT=lpt;108 PE_LAYOUT=lpt;116 PE_LAYOUT=lpt;100 PE_LAYOUT=lpt" timeout -k 10 240 python -u tools/layout_probe.py > $O/r4_ti48c.txt 2>&1 || { tail $O/r4_ti48c.txt; exit 1; }
cat $O/r4_ti48c.txt
echo EXIT 0

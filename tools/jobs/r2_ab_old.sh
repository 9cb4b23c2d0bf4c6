# A/B on one box: the session-start build (_ab/pe_hip_old) vs the current bin/pe_hip.
cd $GRAFT_REPO_ROOT
for r in 1 2; do
 for b in _ab/pe_hip_old bin/pe_hip; do
  for g in "1600 2400" "2400 3200" "8192 8192"; do
   timeout -k 10 60 $b --json $g 2>/dev/null | tail -1 | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); print('$b', d['M'], d['N'], d['iters'], 'T_solver %.4f construct %.4f us/it %.1f' % (d['t_solver'], d['t_construct'], 1e6*d['t_iterate']/d['iters']))" || exit 1
  done
 done
done
PROBE_CFG=8:device timeout -k 10 100 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1

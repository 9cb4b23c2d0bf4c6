# A/B with fixed rows per item (no tuning noise): session-start build vs current.
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
 for b in _ab/pe_hip_old bin/pe_hip; do
  for g in "1600 2400" "2400 3200"; do
   PE_TI=14 PE_TI_TUNE=0 timeout -k 10 60 $b --json $g 2>/dev/null | tail -1 | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); print('$b', d['M'], d['N'], d['iters'], 'us/it %.1f gpu/it %.1f copy %.4f samples %d' % (1e6*d['t_iterate']/d['iters'], 1e6*d['t_gpu']/d['iters'], d['t_copy'], d['timer_samples']))" || exit 1
  done
 done
done

# A/B on one box: per-chunk state read by copy kernel (default) vs hipMemcpyAsync.
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
 for m in kernel memcpy; do
  for g in "1600 2400" "2400 3200"; do
   PE_STATE_COPY=$m timeout -k 10 60 bin/pe_hip --json $g 2>/dev/null | tail -1 | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); print('$m', d['M'], d['N'], d['iters'], 'T_solver %.4f construct %.4f us/it %.1f' % (d['t_solver'], d['t_construct'], 1e6*d['t_iterate']/d['iters']))" || exit 1
  done
 done
done

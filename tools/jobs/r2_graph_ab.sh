# T_solver / loop time: chunk graphs vs eager launches, with and without the
# construction warm-up copy (fresh process per run).
cd $GRAFT_REPO_ROOT
for r in 1 2; do
 for cfg in "0 1" "1 1" "0 0" "1 0"; do
  set -- $cfg   # no-graph? warm-copy?
  flag=""; [ $1 = 1 ] && flag="--no-graph"
  for g in "1600 2400" "2400 3200" "8192 8192"; do
   PE_WARM_COPY=$2 timeout -k 10 60 bin/pe_hip --json $flag $g 2>/dev/null | tail -1 | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); print('nograph=$1 warm=$2', d['M'], d['N'], d['iters'], 'T_solver %.4f construct %.4f us/it %.1f gpu/it %.1f' % (d['t_solver'], d['t_construct'], 1e6*d['t_iterate']/d['iters'], 1e6*d['t_gpu']/d['iters']))" || exit 1
  done
 done
done

cd $GRAFT_REPO_ROOT
for r in 1 2; do
 for b in "_ab/pe_hip_old 0" "bin/pe_hip 0" "bin/pe_hip 1"; do
  set -- $b
  for g in "1600 2400" "2400 3200"; do
   PE_WARM_COPY=$2 PE_TI=14 PE_TI_TUNE=0 timeout -k 10 60 $1 --json $g 2>/dev/null | tail -1 | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); print('$1 warm=$2', d['M'], d['N'], d['iters'], 'us/it %.1f gpu/it %.1f T_solver %.4f' % (1e6*d['t_iterate']/d['iters'], 1e6*d['t_gpu']/d['iters'], d['t_solver']))" || exit 1
  done
 done
done

# 16384^2 full solve with the default rows per item (fresh process) + 8192^2 unchanged check
set -o pipefail
cd $GRAFT_REPO_ROOT
for g in "16384 16384" "8192 8192"; do
  set -- $g
  timeout -k 10 200 bin/pe_hip --json $1 $2 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1x$2', d['algo'], d['iters'], 'T_solver %.4f' % d['t_solver'], 'iter/s %.1f' % (d['iters']/d['t_iterate']), 'L2 %.4e' % d['l2_err'])" || exit 1
done
echo EXIT 0

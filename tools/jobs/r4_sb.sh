# kS3 scheduling: the steady groups without the stage-level sched_barriers
# (pe_hip_nosb) and without any (pe_hip_nosb2) vs the default, alternating
# fresh processes at 8192^2 (3000 iterations, tol off), with each variant's
# 2048^2 iteration count (golden 1730) -> profiles/r4_xd.txt (appended)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
for b in pe_hip_nosb pe_hip_nosb2; do
  timeout -k 10 60 bin/$b --json --quiet 2048 2048 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b 2048^2 iters', d['iters'], 'res_gap', d['res_gap'])"
done
for i in 1 2 3; do
  for b in pe_hip pe_hip_nosb pe_hip_nosb2; do
    timeout -k 10 60 bin/$b --json --quiet --max-iter 3000 --no-tol 8192 8192 > $O/sb_${b}_${i}.json 2>&1 || { cat $O/sb_${b}_${i}.json; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('$O/sb_${b}_${i}.json') if l.startswith('{')][0]
print('$b run $i', 'iterate %.4f s' % d['t_iterate'], 'us/iter %.1f' % (d['t_iterate'] / d['iters'] * 1e6))"
  done
done
echo EXIT 0

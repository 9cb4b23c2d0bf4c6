# kS3 prefetch depth: 3 rows of r / p loads in flight (default) vs 6
# (pe_hip_xd6: -DPE_S3_XD=6; the depth must divide the 6-step group),
# alternating fresh processes at 8192^2 (3000 iterations, tol off), with
# pe_hip_xd6's 2048^2 iteration count (golden 1730); three-step / residual
# GPU tests at the default -> profiles/r4_xd.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 200 --timeout-method thread tests/test_three_step.py tests/test_residual.py > $O/r4_xd_tests.txt 2>&1 || { tail -30 $O/r4_xd_tests.txt; exit 1; }
tail -1 $O/r4_xd_tests.txt
for i in 1 2 3; do
  for b in pe_hip pe_hip_xd6; do
    timeout -k 10 60 bin/$b --json --quiet --max-iter 3000 --no-tol 8192 8192 > $O/xd_${b}_${i}.json 2>&1 || { cat $O/xd_${b}_${i}.json; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('$O/xd_${b}_${i}.json') if l.startswith('{')][0]
print('$b run $i', 'iterate %.4f s' % d['t_iterate'], 'us/iter %.1f' % (d['t_iterate'] / d['iters'] * 1e6))"
  done
done
timeout -k 10 60 bin/pe_hip_xd6 --json --quiet 2048 2048 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('xd6 2048^2 iters', d['iters'], 'res_gap', d['res_gap'])"
echo EXIT 0

# Last-round pool of the three-step static list (PE_POOL3=1: a block's 4
# last-round items go to whichever of its waves asks first; deterministic
# slot sums): three-step / residual / layout GPU tests with it on, pool on/off
# at one placement (tools/layout_probe.py: 8192^2, 16384^2; block_probe for the
# rank blocks), and the kernel without the pool code (pe_hip_head) vs the new
# build with the pool off, fresh processes -> profiles/r4_pool.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PE_POOL3=1 timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 200 --timeout-method thread tests/test_three_step.py tests/test_residual.py tests/test_layout.py > $O/r4_pool_tests.txt 2>&1 || { tail -30 $O/r4_pool_tests.txt; exit 1; }
tail -1 $O/r4_pool_tests.txt
{
PROBE_P=1 PROBE_ROUNDS=3 PROBE_CFGS="112;112 PE_POOL3=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_GRID=16384x16384 PROBE_ITERS=120 PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="448;448 PE_POOL3=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_P=8 PROBE_ROUNDS=2 PROBE_CFGS="64;64 PE_POOL3=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_P=4 PROBE_ROUNDS=2 PROBE_CFGS="90;90 PE_POOL3=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
} > $O/r4_pool.txt 2>&1 || { tail -20 $O/r4_pool.txt; exit 1; }
grep -v amdgpu.ids $O/r4_pool.txt
for i in 1 2; do
  for b in pe_hip_head pe_hip; do
    timeout -k 10 60 bin/$b --json --quiet --max-iter 3000 --no-tol 8192 8192 > $O/pool_${b}_${i}.json 2>&1 || { cat $O/pool_${b}_${i}.json; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('$O/pool_${b}_${i}.json') if l.startswith('{')][0]
print('$b run $i', 'us/iter %.1f' % (d['t_iterate'] / d['iters'] * 1e6))"
  done
done
echo EXIT 0

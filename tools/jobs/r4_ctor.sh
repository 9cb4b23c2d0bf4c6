# Construction cost of the tuned blocks after the shorter rows-per-item
# timing (S_0 + 1 + 4 sweeps per candidate) and the reused list buffer:
# published grids in fresh processes (PE_CTOR_TRACE=1), the tuned picks of
# the multi-rank blocks (tools/block_probe.py) -> profiles/r4_ctor.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4ctor; mkdir -p $O
for g in "1600 2400" "2400 3200" "2048 2048" "4096 4096"; do
  f=$O/g_${g/ /x}.json
  PE_CTOR_TRACE=1 timeout -k 10 120 bin/pe_hip --json --quiet $g > $f 2>&1 || { cat $f; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$g', d['algo'], d['iters'], 'T_solver %.4f' % d['t_solver'], 'construct %.4f' % d['t_construct'], 'iterate %.4f' % d['t_iterate'])"
  grep "tuning" $f
done
PROBE_CFG=8:device,4:device,2:device,8:4x2 timeout -k 10 300 python3 -u tools/block_probe.py > $O/block.txt 2>&1 || { tail $O/block.txt; exit 1; }
grep -v amdgpu.ids $O/block.txt
echo EXIT 0

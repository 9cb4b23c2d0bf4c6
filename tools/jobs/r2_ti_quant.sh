# Rows-per-item candidates that quantise items per wave (2..5): block probe of
# 8/4/2-rank 8192^2 blocks, the static-layout published grids, and the stamp timeline of the 8-rank block.
cd $GRAFT_REPO_ROOT
PROBE_CFG=8:device,4:device,2:device timeout -k 10 200 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_CFG=1:device PROBE_GRID=2400x3200 timeout -k 10 100 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_CFG=1:device PROBE_GRID=1600x2400 timeout -k 10 100 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_CFG=1:device PROBE_GRID=4096x4096 timeout -k 10 100 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
for g in "1600 2400" "2400 3200" "2048 2048" "4096 4096"; do
  timeout -k 10 60 bin/pe_hip --json $g 2>/dev/null | tail -1 | python3 -c "
import sys, json; d=json.loads(sys.stdin.read()); print(d['M'], d['N'], d['iters'], 'T_solver %.4f construct %.4f us/it %.1f' % (d['t_solver'], d['t_construct'], 1e6*d['t_iterate']/d['iters']))" || exit 1
done
PROBE_CFG=8:device timeout -k 10 120 python3 -u tools/stamp_probe.py 2>&1 | grep -E "span|busy fraction|wave exit|item duration" | head -8

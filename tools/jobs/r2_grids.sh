# Round 2: published + BASELINE grids, full solves (bin/pe_hip --json: T_solver incl.
# construction, sampled per-phase timers; first process on the box runs 400x600),
# a construction-phase trace of 800x1200, then the 8/4/2-rank block probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/grids; mkdir -p $O
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "800 1200"; do
  timeout -k 10 90 bin/pe_hip --json $g > $O/g_${g/ /x}.json 2>&1 || { cat $O/g_${g/ /x}.json; exit 1; }
  tail -1 $O/g_${g/ /x}.json
done
PE_CTOR_TRACE=1 timeout -k 10 60 bin/pe_hip --json 800 1200 2>&1 | grep "ctor" || exit 1
PROBE_CFG=8:device,4:device,2:device timeout -k 10 200 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
echo EXIT 0

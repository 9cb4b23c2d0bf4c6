# Round 2 validation: GPU suite, published/BASELINE grids (fresh processes),
# 8/4/2-rank block probe, bench short and long.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  timeout -k 10 120 bin/pe_hip --json $g > $O/g_${g/ /x}.json 2>&1 || { cat $O/g_${g/ /x}.json; exit 1; }
  tail -1 $O/g_${g/ /x}.json
done
PROBE_CFG=8:device,4:device,2:device timeout -k 10 200 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
cat $O/bench20.json
timeout -k 10 120 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || exit 1
cat $O/bench2000.json
echo EXIT 0

# Round 2 quick check: golden-count GPU tests, full solves of the key grids, 8-rank block, 8192^2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/quick; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "golden or oracle or virtual or thin or classic_state or deterministic or odd_conv" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest.txt | head -20; exit $rc; }
for g in "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192"; do
  r=$(timeout -k 10 60 $BIN --json --quiet $g) || exit 1
  echo "$g $(echo $r | grep -o '"iters": [0-9]*'), $(echo $r | grep -o '"t_iterate": [0-9.]*')"
done
PROBE_CFG=8:device timeout -k 10 120 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_GRID=800x1200 PROBE_CFG=1:aspect timeout -k 10 120 python3 -u tools/stamp_probe.py > $O/stamp_800.txt 2>&1 || exit 1
grep -E "span|item duration|band items|busy fraction|us/iter|after row step|prologue|item end" $O/stamp_800.txt | head -40
echo EXIT 0

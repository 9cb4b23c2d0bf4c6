# Round 2: small / medium block tuning (full solves; rows per item, heavy-item split) + the 8-rank block.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/tune; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
for g in "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096"; do
  for v in "PE_TI=8" "PE_TI=8 PE_HEAVY_SPLIT=0" "PE_TI=6" "PE_TI=4" "PE_TI=12"; do
    r=$(env $v timeout -k 10 60 $BIN --json --quiet $g) || exit 1
    echo "$g [$v] $(echo $r | grep -o '"iters": [0-9]*'), $(echo $r | grep -o '"t_iterate": [0-9.]*')"
  done
done
for v in "PE_TI=8" "PE_TI=6" "PE_TI=4" "PE_TI=8 PE_HEAVY_SPLIT=0"; do
  PROBE_CFG=8:device PROBE_ENV="$v" timeout -k 10 120 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
PROBE_GRID=800x1200 PROBE_CFG=1:aspect timeout -k 10 120 python3 -u tools/stamp_probe.py > $O/stamp_800.txt 2>&1 || exit 1
grep -E "span|item duration|band items|busy fraction|us/iter" $O/stamp_800.txt
echo EXIT 0

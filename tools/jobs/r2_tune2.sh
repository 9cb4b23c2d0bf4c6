# Round 2: grid timings under item-size / split variants (full solves, t_iterate).
set -o pipefail
cd $GRAFT_REPO_ROOT
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
run() { local g="$1"; shift; r=$(env "$@" timeout -k 10 60 $BIN --json --quiet $g) || exit 1; echo "$g [$*] $(echo $r | grep -o '"iters": [0-9]*'), $(echo $r | grep -o '"t_iterate": [0-9.]*')"; }
for v in "PE_TI=16" "PE_TI=14" "PE_TI=18"; do run "8192 8192" $v; done
for g in "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096"; do
  for v in "PE_TI=8" "PE_TI=8 PE_HEAVY_SPLIT=0" "PE_TI=6" "PE_TI=10"; do run "$g" $v; done
done
PROBE_CFG=8:device PROBE_ENV="PE_TI=8;PE_TI=6;PE_TI=10;PE_TI=8 PE_HEAVY_SPLIT=0" timeout -k 10 120 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
echo EXIT 0

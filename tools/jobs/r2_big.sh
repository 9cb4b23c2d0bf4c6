# Round 2: 8192^2 / 16384^2 rows-per-item sweep, two runs each (placement noise).
set -o pipefail
cd $GRAFT_REPO_ROOT
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
run() { local g="$1"; shift; r=$(env "$@" timeout -k 10 90 $BIN --json --quiet $g) || exit 1; echo "$g [$*] $(echo $r | grep -o '"iters": [0-9]*'), $(echo $r | grep -o '"t_iterate": [0-9.]*')"; }
for v in "PE_TI=16" "PE_TI=18" "PE_TI=14" "PE_TI=22" "PE_TI=16" "PE_TI=18" "PE_TI=14" "PE_TI=22"; do run "8192 8192" $v; done
for v in "PE_TI=16" "PE_TI=18"; do run "16384 16384" $v; done
for g in "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096"; do run "$g" PE_X=1; done
echo EXIT 0

set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/check2; mkdir -p $O
run() { timeout -k 10 200 ./bin/pe_hip --json "$@" 2>&1 | grep '^{' ; }
( for g in "40 40" "10 10" "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048"; do run $g || exit 1; done
  run --variant 1 400 600 && run --variant 1 800 1200 && run --variant 1 2048 2048 &&
  for v in 2 3 4 6 8; do run --vranks $v 400 600 || exit 1; done
  run --vranks 8 --decomp reference 800 1200 && run --vranks 5 1600 2400 &&
  run --init random 800 1200 && run 4096 4096 && run 8192 8192 && run --variant 1 8192 8192 ) > $O/res.txt
echo EXIT $?

set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/check3; mkdir -p $O
run() { timeout -k 10 200 ./bin/pe_hip --json "$@" 2>&1 | grep '^{' ; }
( for g in "40 40" "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192"; do run $g || exit 1; done
  run --variant 1 800 1200 && run --variant 1 8192 8192 &&
  for v in 2 3 4 8; do run --vranks $v 400 600 || exit 1; done
  run --vranks 5 1600 2400 && run --init random 800 1200 &&
  for ti in 8 16 32 60; do PE_TI=$ti run --max-iter 300 --no-tol 8192 8192 || exit 1; done ) > $O/res.txt
echo EXIT $?

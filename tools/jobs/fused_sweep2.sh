# Single-sweep kernel: correctness smoke + (order × rows per item) sweep at
# 8192², and the register-pressure experiment (bin/pe_hip_nogen: band rows
# treated as band-free — timing only, its numbers are not a solution).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/fsweep2; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
timeout -k 10 60 $BIN --json --quiet 400 600 > $O/smoke.txt 2>&1 && timeout -k 10 60 $BIN --json --quiet --vranks 9 --decomp aspect 700 500 >> $O/smoke.txt 2>&1 || { echo smoke failed; cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt | cut -c1-160
( for order in 0 2; do for ti in 8 12 16; do
    echo "order=$order ti=$ti"; PE_ORDER=$order PE_TI=$ti timeout -k 10 100 $BIN --json --quiet --max-iter 1000 --no-tol 8192 8192 || exit 1
  done; done
  for ti in 8 16; do echo "nogen ti=$ti"; PE_TI=$ti timeout -k 10 100 ${BIN}_nogen --json --quiet --max-iter 1000 --no-tol 8192 8192 || exit 1; done
  echo "full"; timeout -k 10 100 $BIN --json --quiet 8192 8192 || exit 1
) > $O/sweep.txt 2>&1 || { echo sweep failed; tail $O/sweep.txt; exit 1; }
grep -E "order=|nogen|full|iters_per_s" $O/sweep.txt | paste - - | sed -E 's/\{.*"iters": ([0-9]+).*"iters_per_s": ([0-9.]+).*"l2_err": ([0-9.e+-]+).*/iters=\1 ips=\2 l2=\3/'

# Single-sweep kernel configurations (PE_SKERNEL: 0 default, 1 non-temporal
# streams, 2 prefetch depth 3, 3 both) × rows per item at 8192².
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/fsweep3; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
timeout -k 10 60 $BIN --json --quiet 400 600 > $O/smoke.txt 2>&1 || { echo smoke failed; cat $O/smoke.txt; exit 1; }
cut -c1-120 $O/smoke.txt
( for cfg in 3 4 5 6; do for ti in 8 16 32; do
    echo "cfg=$cfg ti=$ti"; PE_SKERNEL=$cfg PE_TI=$ti timeout -k 10 100 $BIN --json --quiet --max-iter 1000 --no-tol 8192 8192 || exit 1
  done; done
) > $O/sweep.txt 2>&1 || { echo sweep failed; tail $O/sweep.txt; exit 1; }
grep -E "cfg=|iters_per_s" $O/sweep.txt | paste - - | sed -E 's/\{.*"iters": ([0-9]+).*"iters_per_s": ([0-9.]+).*/iters=\1 ips=\2/'

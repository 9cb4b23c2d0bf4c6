# Full solves (tol 1e-6, w0 = 0) of the published and BASELINE grids on one GPU with the default
# single-sweep path, plus the per-phase timer breakdown at 8192² and 16384².
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/grids; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
for g in "200 200" "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  echo "== $g"; timeout -k 10 120 $BIN --json $g > $O/g_${g/ /x}.json 2> $O/g_${g/ /x}.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k] for k in d if k in ('iters','t_solver','iters_per_s','l2_err','converged','status','timers')})" $O/g_${g/ /x}.json || cat $O/g_${g/ /x}.json
done
echo "== timing 8192"; timeout -k 10 120 $BIN --timing 8192 8192 > $O/timing_8192.txt 2>&1 || exit 1; cat $O/timing_8192.txt
echo "== timing 16384"; timeout -k 10 200 $BIN --timing 16384 16384 > $O/timing_16384.txt 2>&1 || exit 1; cat $O/timing_16384.txt

# Round 3: two-step sweep (fused2.hip) — tests, then bench 8192^2 two-step vs single sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3two; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_two_step.py -v --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.txt 2>&1; rc=$?
tail -30 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for algo in two-step fused two-step fused; do
  timeout -k 10 150 python -u bench.py --algo $algo --steps 400 --warmup 40 --no-random-solve > $O/bench_$algo.json 2> $O/bench_$algo.err || { tail $O/bench_$algo.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$algo.json')); print('$algo', round(d['value'],1), d['ms_per_step'], d['iters_converged'], d['l2_err'], d['config']['placement']['candidates_ms_per_sweep'], d['t_solver_s'])"
done
echo EXIT 0

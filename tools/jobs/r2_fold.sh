# Item-sum fold: targeted GPU tests, then bench with fold on / off (PE_FOLD=0) and a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/fold; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "fold or item_orders or golden or fault or multi_process_2d or halo_push" > $O/pytest.txt 2>&1; rc=$?
tail -5 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
for f in 1 0 1 0; do
  PE_FOLD=$f timeout -k 10 120 python -u bench.py --steps 2000 --warmup 50 --no-solve > $O/bench_fold$f.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_fold$f.json')); print('fold $f', round(d['value'],1), d['config']['placement'])"
done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/bench20.json')); print('steps 20:', round(d['value'],1), d['t_solver_s'], d['iters_converged'], d['l2_err'])"
echo EXIT 0

# Round 3: GPU test suite (new tests first), driver smoke, short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3suite; mkdir -p $O
K="${PYTEST_K:-}"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -v --timeout 120 --timeout-method thread \
  -k "self_launch or stalled or slow_rank or resident_barrier or terminal_at_launch or forced_breakdown or graft_smoke" > $O/new.txt 2>&1; rc=$?
tail -15 $O/new.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -8 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
cat $O/bench20.json
echo EXIT 0

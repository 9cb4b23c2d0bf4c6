# Round 3: full GPU suite, smoke, short and long bench (default algorithm).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3suite3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.txt 2>&1; rc=$?
tail -12 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || { tail $O/bench2000.err; exit 1; }
cat $O/bench2000.json
echo EXIT 0

# Round 3: full GPU suite, smoke, bench (default two-step), rows-per-item probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3suite2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.txt 2>&1; rc=$?
tail -12 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
cat $O/bench20.json
PROBE_GRIDS=1600x2400,2048x2048,4096x4096,8192x8192,16384x16384 PROBE_TI=16,24,32,40,48 PROBE_ITERS=200 \
  timeout -k 10 400 python -u tools/ti_probe.py > $O/ti_probe.txt 2>&1 || { tail $O/ti_probe.txt; exit 1; }
grep -v amdgpu.ids $O/ti_probe.txt
echo EXIT 0

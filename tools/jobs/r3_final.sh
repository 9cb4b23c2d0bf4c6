# Round 3 validation at HEAD: full GPU suite, driver smoke, driver-shaped and
# long bench; then one rank's 2-D block timed single sweep vs three-step
# (tools/block_probe.py) and the short-window probe (tools/window_probe.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r3final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -12 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || { tail $O/bench2000.err; exit 1; }
cat $O/bench2000.json
PROBE_CFG=8:4x2,4:2x2,8:rows PROBE_ENV="PE_STEPS=1;PE_STEPS=3" timeout -k 10 300 python3 -u tools/block_probe.py > $O/block.txt 2>&1 || { tail $O/block.txt; exit 1; }
cat $O/block.txt
timeout -k 10 150 python3 -u tools/window_probe.py > $O/window.txt 2>&1 || { tail $O/window.txt; exit 1; }
cat $O/window.txt
echo EXIT 0

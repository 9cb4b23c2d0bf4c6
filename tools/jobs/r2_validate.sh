# Round 2 validation: GPU test suite, bench (short and long), published grids
# with the per-phase timer breakdown (bin/pe_hip --json).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/validate; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -5 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
cat $O/bench20.json
timeout -k 10 120 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || exit 1
cat $O/bench2000.json
for g in "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192"; do
  timeout -k 10 60 bin/pe_hip --json $g > $O/grid_${g/ /x}.json || exit 1
  tail -1 $O/grid_${g/ /x}.json
done
timeout -k 10 60 bin/pe_hip 800 1200 > $O/legacy_800.txt || exit 1
cat $O/legacy_800.txt
echo EXIT 0

# Round 6, first GPU call: baseline at HEAD (start of round) — GPU test suite
# and the driver-shaped bench (20 steps), plus a 2-rank / 8-rank slab probe.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6first; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt
echo EXIT 0

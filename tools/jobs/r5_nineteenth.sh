# Round 5, nineteenth GPU call: the whole GPU suite after the n-major reduction in every sweep, the tuner finalists, the new layout / priority tests
# (single / two-step sweeps too)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5nineteenth; mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -5 $O/gpu_tests.txt
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
exit $rc

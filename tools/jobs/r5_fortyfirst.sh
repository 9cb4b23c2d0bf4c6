# Round 5, forty-first GPU call: the whole GPU suite with the exchange as the row slabs. default (push opt-in)
# (stop tests, fix-up, breakdown / cap, restart paths all read the snapshot)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fortyfirst; mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -5 $O/gpu_tests.txt
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
exit $rc

# Round 5, thirty-fourth GPU call: the whole GPU suite at the round-5 final HEAD (finalize scalars in LDS)
# (stop tests, fix-up, breakdown / cap, restart paths all read the snapshot)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirtyfourth; mkdir -p $O
cd $R
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -5 $O/gpu_tests.txt
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
exit $rc

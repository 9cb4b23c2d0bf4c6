# First device run of the single-sweep kernel: small goldens, the headline
# grid, then the GPU test suite.  Every step is time-limited; stop at the
# first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fused1; mkdir -p $O
run() { echo "== $*" >> $O/apps.txt; timeout -k 10 120 "$@" >> $O/apps.txt 2>&1; }
run bin/pe_hip --algo fused 40 40 && run bin/pe_hip --algo fused 400 600 && \
run bin/pe_hip --algo fused --vranks 4 400 600 && run bin/pe_hip --algo fused 8192 8192 && \
run bin/pe_hip --algo classic 8192 8192
rc=$?
cat $O/apps.txt | grep -E "==|iter|Iter|L2|error|rror|time|Time" | head -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest.txt 2>&1
rc=$?
tail -15 $O/pytest.txt
exit $rc

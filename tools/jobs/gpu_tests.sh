set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gputest; mkdir -p $O
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest.txt 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest.txt
[ $rc -eq 0 ] && timeout -k 10 300 python bench.py > $O/bench.txt 2> $O/bench.err && cat $O/bench.txt
echo EXIT $?

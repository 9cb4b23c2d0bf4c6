# Full GPU check: test suite, headline bench, kernel-trace profile at 8192².
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/check; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- $GRAFT_REPO_ROOT/bin/pe_hip --quiet --max-iter 300 --no-tol 8192 8192 > $O/kt.log 2>&1
echo EXIT $?

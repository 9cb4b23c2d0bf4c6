set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/check5; mkdir -p $O
timeout -k 10 1000 python -m pytest tests -m gpu -x -q > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 bin/pe_hip --json --quiet 16384 16384 > $O/big.txt 2>&1 || { tail $O/big.txt; exit 1; }
cut -c1-400 $O/big.txt

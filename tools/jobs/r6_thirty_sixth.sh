# Round 6, thirty-sixth GPU call: the halo choice agrees on the number of
# overlap heights across ranks (each rank tunes its own block) — the new
# 2-process test with one tuned and one untuned rank, then the host-staged
# multi-process matrix.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirtysixth; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py -m gpu -k "agrees or multi_process" > $O/t.txt 2>&1 || { tail -40 $O/t.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/t.txt | tail -20
echo EXIT 0

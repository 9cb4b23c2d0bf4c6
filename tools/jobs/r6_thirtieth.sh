# Round 6, thirtieth GPU call: the filling layout stops once its passes
# repeat; untraced fresh-process grids for the tables (T_solver with the
# pipelined tuning), the construction trace of the halo choice, the layout /
# halo / overlap GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirtieth; mkdir -p $O
cd $R
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  timeout -k 10 150 bin/pe_hip --json $g > $O/grid_${g/ /x}.json 2> $O/grid_${g/ /x}.err || { tail -5 $O/grid_${g/ /x}.err; exit 1; }
  echo "grid $g done"
done
PE_CTOR_TRACE=3 timeout -k 10 200 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -20 $O/ctor.txt; exit 1; }
grep -E "construction" $O/ctor.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_layout.py tests/test_gpu.py -m gpu -k "layout or tun or halo_path or overlap or resume" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
echo EXIT 0

# Round 6, twenty-eighth GPU call: the rows-per-item tuning pipelined (host
# layout of trial i+1 under the GPU timing of trial i, cached layouts) —
# construction phases and layout laps on the small / mid grids, then the
# layout / tuning GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twentyeighth; mkdir -p $O
cd $R
for g in "2048 2048" "1600 2400" "2400 3200" "4096 4096"; do
  PE_CTOR_TRACE=3 timeout -k 10 120 bin/pe_hip --json $g > $O/grid_${g/ /x}.json 2> $O/grid_${g/ /x}.err || { tail -5 $O/grid_${g/ /x}.err; exit 1; }
  echo "== $g"; grep -E "ctor|layout (lpt|equal|fill|list)|equal:" $O/grid_${g/ /x}.err | head -80
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_layout.py tests/test_gpu.py -m gpu -k "layout or tun or halo_path or overlap or resume" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
echo EXIT 0

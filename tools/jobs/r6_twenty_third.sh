# Round 6, twenty-third GPU call: the published and BASELINE grids at HEAD
# (bin/pe_hip --json, one fresh process per grid) and the 2000-step bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twentythird; mkdir -p $O
cd $R
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  timeout -k 10 150 bin/pe_hip --json $g > $O/grid_${g/ /x}.json 2> $O/grid_${g/ /x}.err || { tail -5 $O/grid_${g/ /x}.err; exit 1; }
  echo "grid $g done"
done
timeout -k 10 200 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || { tail -5 $O/bench2000.err; exit 1; }
tail -1 $O/bench2000.json | cut -c1-200
echo EXIT 0

# Round 6, twenty-ninth GPU call: HEAD with the pipelined rows-per-item tuning
# and cached equal-cost runs — the published / BASELINE grids (fresh process
# each, construction phases traced), smoke, the whole GPU suite, the bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twentyninth; mkdir -p $O
cd $R
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  PE_CTOR_TRACE=1 timeout -k 10 150 bin/pe_hip --json $g > $O/grid_${g/ /x}.json 2> $O/grid_${g/ /x}.err || { tail -5 $O/grid_${g/ /x}.err; exit 1; }
  echo "grid $g: $(grep 'ctor ti tuning' $O/grid_${g/ /x}.err)"
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.txt').read().strip().splitlines()[-1]);print('bench',round(d['value'],1),d['t_solver_s'],d['iters_converged'],d['l2_err'])"
echo EXIT 0

# Round 6, forty-seventh GPU call: the placement search on the 2-rank block of
# 8192² with the 24-50 M-node stop rate (4.0 TB/s) and no retry round below
# 50 M nodes — one fresh process per construction; then the 1-GPU bench
# (8192², unchanged rule) once.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fortyseventh; mkdir -p $O
cd $R
for i in 1 2 3; do
  PROBE_CFG=2:rows PROBE_REPS=1 timeout -k 10 200 python -u tools/placement_probe.py > $O/p_$i.txt 2>&1 || { tail -20 $O/p_$i.txt; exit 1; }
  grep "^P=" $O/p_$i.txt | cut -c1-400
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.txt').read().strip().splitlines()[-1]);p=d['config']['placement'];print('bench',round(d['value'],1),p['candidates_ms_per_sweep'],p['search_s'],round(d['t_solver_s'],4))"
echo EXIT 0

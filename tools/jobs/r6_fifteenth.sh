# Round 6, fifteenth GPU call: the whole GPU suite and smoke at HEAD (put /
# P2P-sum fence changes), the 1-GPU bench, the halo probe at 15/8 and 60/8.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fifteenth; mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.txt').read().strip().splitlines()[-1]);print('bench',round(d['value'],1),d['t_solver_s'],d['iters_converged'],d['l2_err'])"
PROBE_CFG=8:rows,8:4x2 PROBE_ITERS=300 timeout -k 10 300 python -u tools/halo_probe.py 15 8 60 8 > $O/halo_probe.txt 2>&1 || { tail -20 $O/halo_probe.txt; exit 1; }
grep -v amdgpu.ids $O/halo_probe.txt
echo EXIT 0

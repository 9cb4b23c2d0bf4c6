# Round 6, forty-eighth GPU call: the whole GPU suite and smoke at the final HEAD (the
# placement stop rates by block size, no retry below 50 M nodes), the 1-GPU bench (two fresh processes),
# the construction trace, the halo probe at 0/0 and 15/8.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fortyeighth; mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
PE_CTOR_TRACE=3 timeout -k 10 200 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -20 $O/ctor.txt; exit 1; }
grep -E "halo path (reset|re-layout|.*apply)|construction" $O/ctor.txt > $O/ctor_short.txt; grep construction $O/ctor_short.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_$i.txt 2>&1 || { tail -20 $O/bench_$i.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$i.txt').read().strip().splitlines()[-1]);print('bench',round(d['value'],1),d['t_solver_s'],d['iters_converged'],d['l2_err'],d['config']['placement']['candidates_ms_per_sweep'])"
done
PROBE_HALO=exchange timeout -k 10 400 python -u tools/halo_probe.py 0 0 15 8 > $O/proj.txt 2>&1 || { tail -20 $O/proj.txt; exit 1; }
grep -v amdgpu.ids $O/proj.txt | cut -c1-200
echo EXIT 0

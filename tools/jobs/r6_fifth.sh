# Round 6, fifth GPU call: same-box A/B of the 1-GPU bench (HEAD vs the
# round-5 build in .r5ref, alternating fresh processes), the 2-D three-step
# multi-process tests (the 6-process put+overlap stall), the put's local cost.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fifth; mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/head_$i.txt 2>&1 || { tail -20 $O/head_$i.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/head_$i.txt').read().strip().splitlines()[-1]);print('HEAD',round(d['value'],1),d['config']['placement']['candidates_ms_per_sweep'],d['config']['placement']['chosen'])"
  timeout -k 10 200 python -u .r5ref/bench.py --steps 20 --warmup 5 --no-random-solve > $O/r5_$i.txt 2>&1 || { tail -20 $O/r5_$i.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/r5_$i.txt').read().strip().splitlines()[-1]);print('R5  ',round(d['value'],1),d['config']['placement']['candidates_ms_per_sweep'],d['config']['placement']['chosen'])"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py -k "multi_process_2d_three_step" > $O/mp3.txt 2>&1 || { tail -40 $O/mp3.txt; exit 1; }
grep -E "PASSED|FAILED" $O/mp3.txt
PROBE_CFG=8:rows,8:4x2 PROBE_EACH=1 PROBE_ITERS=300 timeout -k 10 300 python -u tools/halo_probe.py 0 0 > $O/halo_probe.txt 2>&1 || { tail -20 $O/halo_probe.txt; exit 1; }
cat $O/halo_probe.txt
echo EXIT 0

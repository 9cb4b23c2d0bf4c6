# Round 5, second GPU call: the band 1/D ring + 4-row item candidates for
# small blocks: three-step tests, block probes (-> profiles/r5_block_probe_b.txt),
# stamped timelines with the new step / launch stamps (-> profiles/r5_stamps.txt),
# driver-shaped bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5second; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_three_step.py tests/test_layout.py tests/test_residual.py tests/test_gpu.py::test_overlap_async_loopback_transport_bitwise tests/test_gpu.py::test_bench_two_step_warmup_counts > $O/tests.txt 2>&1; rc=$?
tail -5 $O/tests.txt; echo "tests rc $rc"; [ $rc -eq 0 ] || exit 1
PROBE_CFG=2:device,4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe8192.txt 2>&1 || exit 1
PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_CFG=8:device timeout -k 10 240 python -u tools/block_probe.py > $O/probe16384.txt 2>&1 || exit 1
PROBE_GRID=4096x4096 PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe4096.txt 2>&1 || exit 1
for g in 800x1200 1600x2400 2400x3200 2048x2048; do
  PROBE_GRID=$g PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe$g.txt 2>&1 || exit 1
done
grep -h "us/iter" $O/probe*.txt
PROBE_CFG=8:4x2,4:2x2 PROBE_GRAPH=0 timeout -k 10 240 python -u tools/overlap_probe.py 15 8 > $O/overlap.txt 2>&1 || exit 1
grep -h "us/iter" $O/overlap.txt
PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
PROBE_GRID=1600x2400 PROBE_CFG=2:device timeout -k 10 120 python -u tools/stamp_probe.py > $O/stamps1600.txt 2>&1 || { tail -20 $O/stamps1600.txt; exit 1; }
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || exit 1
  PE_LPT_KIND=0 timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-solve > $O/benchk$i.json 2> $O/benchk$i.err || exit 1
done
python3 -c "
import json
for n in ('bench1','benchk1','bench2','benchk2','bench3','benchk3'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); print(n, d['value'], d['ms_per_step'], d.get('iters_converged'), d.get('t_iterate_s'), d.get('t_check_s'))"
# four-step sweep (opt-in): tests, bench, slab / 8192^2 probes
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_four_step.py > $O/tests4.txt 2>&1; rc=$?
tail -5 $O/tests4.txt; echo "tests4 rc $rc"; [ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --algo four-step > $O/bench4_$i.json 2> $O/bench4_$i.err || exit 1; done
python3 -c "
import json
for n in ('bench4_1','bench4_2'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); print(n, d['value'], d['ms_per_step'], d.get('iters_converged'), d.get('t_iterate_s'), d['config'].get('algo'))"
PE_STEPS=4 PROBE_HALO=8 PROBE_CFG=8:device,1:device timeout -k 10 240 python -u tools/stamp_probe.py > $O/stamps4.txt 2>&1 || { tail -20 $O/stamps4.txt; exit 1; }
grep -h "us/iter" $O/stamps4.txt
echo EXIT 0

# Round 5, sixth GPU call: HEAD defaults (round-4 layouts + band 1/D ring +
# entry preload + paired partial loads + overlap short pieces) vs the round-4
# build on one box; per-rank block probes (zero-delay transport launches
# nothing now), overlap probe, stamped slab timeline, GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5sixth; mkdir -p $O
cd $R
for i in 1 2; do
  (cd .r4ref && timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/r4_$i.json 2> $O/r4_$i.err) || { tail -5 $O/r4_$i.err; exit 1; }
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/head_$i.json 2> $O/head_$i.err || { tail -5 $O/head_$i.err; exit 1; }
done
python3 -c "
import json,glob,os
for f in sorted(glob.glob('$O/*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(os.path.basename(f)[:-5], round(d['value'],1), d['config']['placement']['job_ms_per_sweep'], d.get('iters_converged'), d.get('t_solver_s'), d.get('t_iterate_s'), d['config']['ranks'][0]['pci_bus_id'])"
(cd .r4ref && PROBE_CFG=2:device,4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe_r4.txt 2>&1) || exit 1
PROBE_CFG=2:device,4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe_head.txt 2>&1 || exit 1
PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_CFG=2:device,4:device,8:device timeout -k 10 240 python -u tools/block_probe.py > $O/probe_head16k.txt 2>&1 || exit 1
for g in 4096x4096 1600x2400 2048x2048 2400x3200 800x1200; do
  PROBE_GRID=$g PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe_head_$g.txt 2>&1 || exit 1
done
for f in $O/probe_*.txt; do echo "== $(basename $f)"; grep -h "us/iter" $f; done
PROBE_CFG=8:4x2,4:2x2 PROBE_GRAPH=0 timeout -k 10 240 python -u tools/overlap_probe.py 15 8 > $O/overlap.txt 2>&1 || exit 1
grep -h "us/iter" $O/overlap.txt
PROBE_CFG=8:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || exit 1
grep -h "us/iter\|busy fraction\|tail (max\|gap after\|walk entry\|finalized\|kind " $O/stamps.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_three_step.py tests/test_layout.py tests/test_residual.py tests/test_four_step.py tests/test_gpu.py::test_overlap_async_loopback_transport_bitwise > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; echo "tests rc $rc"; [ $rc -eq 0 ] || exit 1
echo EXIT 0

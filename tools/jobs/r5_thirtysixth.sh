# Round 5, thirty-sixth GPU call: the halo-push kernel without the per-item
# system-scope release (L2 write-back) — per-rank loopback probes, then the
# whole GPU suite (the multi-process push / P2P tests check delivery).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirtysixth; mkdir -p $O
cd $R
for lb in 1 0; do
  PE_PUSH_LOOPBACK=$lb PROBE_CFG=8:device,4:device,2:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/loopback $lb /"
done
PE_PUSH_LOOPBACK=1 PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_CFG=8:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/loopback 1 /"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -3 $O/gpu_tests.txt
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
exit $rc

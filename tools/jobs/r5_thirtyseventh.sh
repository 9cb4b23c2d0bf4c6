# Round 5, thirty-seventh GPU call: the halo-push kernel with its receive-
# buffer pointers read only on the pushing rows (no scalar load per row step)
# — loopback per-rank probes against the plain kernel, then the push / P2P
# multi-process tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirtyseventh; mkdir -p $O
cd $R
for lb in 1 0; do
  PE_PUSH_LOOPBACK=$lb PROBE_CFG=8:device,4:device,2:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/loopback $lb /"
done
PE_PUSH_LOOPBACK=1 PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_CFG=8:device timeout -k 10 200 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/loopback 1 /"
timeout -k 10 600 python -u -m pytest tests/test_multigpu.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "push or p2p or peer or slab or multi or transport or xr" > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt
exit $rc

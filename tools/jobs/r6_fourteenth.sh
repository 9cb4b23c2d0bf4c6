# Round 6, fourteenth GPU call: the put with 16-byte phase-aligned copies —
# correctness (bitwise loopback, host-staged put jobs, checkpoint) and its
# local cost at the 8-rank slab / 4x2 block (halo probe, each path forced).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fourteenth; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py \
  -k "loopback_transport_bitwise or halo_put or env6 or env7" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
grep -E "PASSED|FAILED" $O/tests.txt
PROBE_CFG=8:rows,8:4x2 PROBE_EACH=1 PROBE_ITERS=300 timeout -k 10 300 python -u tools/halo_probe.py 0 0 > $O/halo_probe.txt 2>&1 || { tail -20 $O/halo_probe.txt; exit 1; }
grep -v amdgpu.ids $O/halo_probe.txt
echo EXIT 0

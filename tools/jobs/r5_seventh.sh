# Round 5, seventh GPU call: band-piece cost factor of the equal-cost layout
# (mid-size blocks): PE_COST_BAND 2.45 (default) / 2.8 / 3.1 / 3.4 on the
# 8-rank slab, the 4x2 and 4-rank blocks of 8192^2 and 2-rank blocks of the
# published grids -> profiles/r5_costband.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5seventh; mkdir -p $O
cd $R
for rep in 1 2; do
for cb in 2.45 2.8 3.1 3.4; do
  PE_COST_BAND=$cb PROBE_CFG=8:device,8:4x2,4:device timeout -k 10 200 python -u tools/block_probe.py > $O/p8192_${cb}_$rep.txt 2>&1 || exit 1
  PE_COST_BAND=$cb PROBE_GRID=1600x2400 PROBE_CFG=2:device timeout -k 10 100 python -u tools/block_probe.py > $O/p1600_${cb}_$rep.txt 2>&1 || exit 1
  PE_COST_BAND=$cb PROBE_GRID=2048x2048 PROBE_CFG=1:device timeout -k 10 100 python -u tools/block_probe.py > $O/p2048_${cb}_$rep.txt 2>&1 || exit 1
done
done
for f in $O/p*.txt; do echo "$(basename $f .txt): $(grep -h 'us/iter' $f | sed 's/tuning.*//' | awk '{print $2, $5, $8}' | tr '\n' ' ')"; done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_three_step.py tests/test_layout.py tests/test_residual.py tests/test_four_step.py tests/test_gpu.py::test_overlap_async_loopback_transport_bitwise > $O/tests.txt 2>&1; rc=$?
tail -3 $O/tests.txt; echo "tests rc $rc"; [ $rc -eq 0 ] || exit 1
echo EXIT 0

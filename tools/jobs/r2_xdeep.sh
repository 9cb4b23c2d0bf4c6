# Deferring sweep with 8 x rows in flight (PE_SKERNEL=3) vs 4 (default): correctness subset, headline bench and the 8-rank block, alternating fresh processes.
# (experiment build: kS took an x-prefetch-depth template parameter XD and PE_SKERNEL=3 selected XD=8 for WM=0; reverted after this run)
cd $GRAFT_REPO_ROOT
PE_SKERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "golden_iterations and fused or matches_cpu_oracle or large_golden or item_orders or thin_blocks" 2>&1 | tail -2 || exit 1
for i in 1 2; do
  PE_SKERNEL=3 timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1
  timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1
done
for i in 1 2; do
  PE_SKERNEL=3 PROBE_CFG=8:device,4:device,2:device timeout -k 10 120 python3 -u tools/block_probe.py 2>&1 | grep "^P=" || exit 1
  PROBE_CFG=8:device,4:device,2:device timeout -k 10 120 python3 -u tools/block_probe.py 2>&1 | grep "^P=" || exit 1
done

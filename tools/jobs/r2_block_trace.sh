# Kernel trace of the 8-rank 8192^2 block and 2400x3200 (eager loop): per-kernel durations vs the event-timed iteration -> profiles/r2_block_trace.txt
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
PROBE_CFG=8:device PROBE_ITERS=400 timeout -k 10 120 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/bt8 -o run -- python3 -u tools/block_probe.py || exit 1
PROBE_GRID=2400x3200 PROBE_CFG=1:device PROBE_ITERS=400 timeout -k 10 120 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/bt1 -o run -- python3 -u tools/block_probe.py || exit 1
for d in bt8 bt1; do f=$(ls gpurun_out/$d/*/run_results.db gpurun_out/$d/run_results.db 2>/dev/null | tail -1); echo "== $d $f"; python3 tools/rocpd_summary.py $f --segments 2 --timeline 12 || exit 1; done

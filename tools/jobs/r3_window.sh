# Short timed windows (the driver's 20-step bench shape) on one solver:
# graph vs eager, K = 20 / 18 / 21, with and without an idle gap before the
# window; then the same under a kernel trace (per-sweep durations).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/window; mkdir -p $O
cd $R
timeout -k 10 150 python3 -u tools/window_probe.py || exit 1
echo "== idle 20 ms before each window"
PROBE_IDLE_MS=20 PROBE_K=20 PROBE_REPS=3 timeout -k 10 150 python3 -u tools/window_probe.py || exit 1
cd /tmp && export TMPDIR=/tmp
PROBE_K=20 PROBE_REPS=2 timeout -k 10 150 rocprofv3 --kernel-trace -d $O/kt -o run -- python3 $R/tools/window_probe.py > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
cd $R
db=$(ls $O/kt/run_results.db $O/kt/*/run_results.db 2>/dev/null | tail -1)
python3 tools/rocpd_summary.py $db --timeline 48 || exit 1
echo EXIT 0

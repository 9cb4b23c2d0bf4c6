# Round 6, seventeenth GPU call: which rows-per-item / layout the fresh
# overlapped solvers of the variance probe got (no profiler).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6seventeenth; mkdir -p $O
cd $R
PROBE_REPS=6 timeout -k 10 300 python -u tools/overlap_trace_probe.py > $O/ov.txt 2>&1 || { tail -20 $O/ov.txt; exit 1; }
grep "^rep" $O/ov.txt
echo EXIT 0

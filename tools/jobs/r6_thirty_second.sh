# Round 6, thirty-second GPU call: rocprofv3 kernel traces at HEAD (the overlap
# timed at the tuning's three heights) — fresh solvers with the overlap forced at
# the 8-rank slab, exchange and put; then the 1-GPU bench (per-kernel stats).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirtysecond; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bench -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-random-solve > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ov -o run -- python3 $R/tools/overlap_trace_probe.py > $O/ov.log 2>&1 || { tail -20 $O/ov.log; exit 1; }
grep "^rep" $O/ov.log
PROBE_HALO=put timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ovput -o run -- python3 $R/tools/overlap_trace_probe.py > $O/ovput.log 2>&1 || { tail -20 $O/ovput.log; exit 1; }
grep "^rep" $O/ovput.log
cd $R
for d in bench ov ovput; do
  db=$(ls $O/$d/run_results.db $O/$d/*/run_results.db 2>/dev/null | tail -1)
  echo "== $d ($db)"
  if [ "$d" = bench ]; then python3 tools/rocpd_summary.py $db > $O/$d.summary.txt 2>&1; else python3 tools/rocpd_summary.py $db --segments 5 > $O/$d.summary.txt 2>&1; fi
  head -60 $O/$d.summary.txt
done
echo EXIT 0

# Kernel trace of the driver-shaped bench (--steps 20 --warmup 5): where the
# 20-step window's time goes beyond 20 x the steady per-iteration cost.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/b20; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-solve > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
cd $R
db=$(ls $O/kt/run_results.db $O/kt/*/run_results.db 2>/dev/null | tail -1)
echo "== bench.py --steps 20 --warmup 5 kernel trace ($db)"; python3 tools/rocpd_summary.py $db --timeline 40 || exit 1
grep '^{' $O/kt.log | cut -c1-300 || true
for i in 1 2 3; do
  timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-solve > $O/b$i.json 2> $O/b$i.err || { tail $O/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$i.json')); print('bench20 run $i', round(d['value'],1), 'it/s', round(d['ms_per_step'],4), 'ms/step')"
done
echo EXIT 0

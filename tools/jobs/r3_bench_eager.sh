# bench.py with the eager default: the driver's 20-step shape in 4 fresh processes,
# the bench GPU tests, and one 2000-step run.
set -o pipefail
cd $GRAFT_REPO_ROOT; O=$GRAFT_REPO_ROOT/gpurun_out/beager; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "bench" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4; do
  timeout -k 10 180 python3 -u bench.py --steps 20 --warmup 5 > $O/b$i.json 2> $O/b$i.err || { tail $O/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$i.json')); print('bench20 run $i', round(d['value'],1), 'it/s', round(d['ms_per_step'],4), 'ms/step', d['config']['launch'], 'job', d['config']['placement']['job_ms_per_sweep'])"
done
timeout -k 10 180 python3 -u bench.py --steps 2000 --warmup 100 --no-solve > $O/b2000.json 2> $O/b2000.err || { tail $O/b2000.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b2000.json')); print('bench2000', round(d['value'],1), 'it/s', round(d['ms_per_step'],4), 'ms/step')"
cat $O/b1.json
echo EXIT 0

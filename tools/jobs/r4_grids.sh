# Round 4: published / BASELINE grids, default algorithm, fresh process each
# (T_solver incl. construction, the Table-2 phase breakdown, residual check),
# then the driver-shaped and long bench -> profiles/r4_grids.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r4grids; mkdir -p $O
for g in "400 600" "800 1200" "1600 2400" "2400 3200" "2048 2048" "4096 4096" "8192 8192" "16384 16384"; do
  f=$O/g_${g/ /x}.json
  timeout -k 10 120 bin/pe_hip --json --quiet $g > $f 2>&1 || { cat $f; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$g', d['algo'], d['iters'], 'T_solver %.4f' % d['t_solver'], 'construct %.4f' % d['t_construct'],
      'iterate %.4f' % d['t_iterate'], 'gpu %.4f copy %.4f halo %.4f reduce %.4f dot %.4f' % (d['t_gpu'], d['t_copy'], d['t_halo'], d['t_reduce'], d['t_dot']),
      'L2 %.4e' % d['l2_err'], 'res_gap %.2e' % d['res_gap'], 'restarts %d' % d['restarts'])" || tail -2 $f
done
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/bench2000.json 2> $O/bench2000.err || { tail $O/bench2000.err; exit 1; }
cat $O/bench2000.json
echo EXIT 0

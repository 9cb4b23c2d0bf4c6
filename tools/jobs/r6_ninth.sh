# Round 6, ninth GPU call: the multi-GPU projection table at HEAD (VERDICT r5
# items 2 / 6): one rank's block of every projected split, the exchange arms
# chosen by timing at 0/0 and 15/8 us delays (PROBE_HALO=exchange), 300
# iterations each; the 1-GPU full solves of the same grids for the speedups.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6ninth; mkdir -p $O
cd $R
for g in 800x1200 1600x2400 2400x3200 2048x2048 4096x4096; do
  M=${g%x*}; N=${g#*x}
  timeout -k 10 120 ./bin/pe_hip --json $M $N > $O/one_$g.json 2>> $O/one.err || { tail -5 $O/one.err; exit 1; }
  python -c "import json;d=json.loads([l for l in open('$O/one_$g.json') if l.startswith('{')][0]);print('1GPU $g',d['iters'],'t_solver',d['t_solver'],'t_iterate',d['t_iterate'],'us/it',round(1e6*d['t_iterate']/d['iters'],1))"
done
for spec in "800x1200 2:rows" "1600x2400 2:rows" "2400x3200 2:rows" "2048x2048 2:rows" "4096x4096 2:rows" "8192x8192 2:rows,4:rows,8:rows,8:4x2" "16384x16384 2:rows,4:rows,8:rows"; do
  set -- $spec
  PROBE_GRID=$1 PROBE_CFG=$2 PROBE_HALO=exchange PROBE_ITERS=300 timeout -k 10 300 python -u tools/halo_probe.py 0 0 15 8 >> $O/proj.txt 2>&1 || { tail -20 $O/proj.txt; exit 1; }
done
grep "^P=" $O/proj.txt
echo EXIT 0

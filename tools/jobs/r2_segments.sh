# Segment layout experiment (PE_SEGMENTS=1: one tall equal-cost item per wave, halo rows
# re-read once per segment) vs the default static LPT layout: 8192^2 bench in alternating
# fresh processes (+ full solves: golden count), published grids, 8-rank block -> profiles/r2_segments.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  PE_SEGMENTS=$v timeout -k 10 120 python3 -u bench.py --steps 400 --warmup 20 > gpurun_out/seg_$v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/seg_$v.json')); print('PE_SEGMENTS=$v', round(d['value'],1), 'it/s', round(d['ms_per_step']*1e3,1), 'us/iter  iters', d['iters_converged'], 'l2 %.4e' % d['l2_err'], 'placement', d['config']['placement']['candidates_ms_per_sweep'])" || exit 1
done
for g in "2400 3200" "1600 2400" "4096 4096"; do
  for v in 0 1; do
    PE_SEGMENTS=$v timeout -k 10 60 bin/pe_hip --json $g > gpurun_out/seg_grid.json || exit 1
    echo "PE_SEGMENTS=$v $g $(tail -1 gpurun_out/seg_grid.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('iters', d['iters'], 'us/iter %.1f' % (1e6*d['t_iterate']/d['iters']), 'T_solver %.4f' % d['t_solver'])")"
  done
done
PROBE_CFG=8:device,4:device,2:device PROBE_ENV="PE_SEGMENTS=0;PE_SEGMENTS=1;PE_SEGMENTS=0;PE_SEGMENTS=1" PROBE_ITERS=300 timeout -k 10 300 python3 -u tools/block_probe.py || exit 1
echo EXIT 0

# Round 4 first look: per-item timeline of the three-step sweep (PE_STAMPS=1)
# on 8192^2 and the 8/2-rank row-slab blocks; the end-of-solve true-residual
# check at 2048^2 / 8192^2 (zero and random init) and under the drift fault
# hook; a 600-step bench -> profiles/r4_stamps.txt, profiles/r4_resid.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PROBE_CFG=1:device,8:device,2:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/r4_stamps.txt 2>&1 || { tail -20 $O/r4_stamps.txt; exit 1; }
{
for g in "2048 2048" "8192 8192"; do
  for init in zero random; do
    echo "== $g init $init"; timeout -k 10 120 bin/pe_hip --json --quiet --init $init $g || exit 1
  done
done
echo "== 2048 drift@iter:900,amp:1e-3"
PE_FAULT_INJECT=drift@iter:900,amp:1e-3 timeout -k 10 120 bin/pe_hip --json --quiet 2048 2048 || exit 1
echo "== 2048 --algo fused"; timeout -k 10 120 bin/pe_hip --json --quiet --algo fused 2048 2048 || exit 1
} > $O/r4_resid.txt 2>&1 || { tail -20 $O/r4_resid.txt; exit 1; }
timeout -k 10 200 python -u bench.py --steps 600 --warmup 20 > $O/r4_bench600.txt 2>&1 || { tail -20 $O/r4_bench600.txt; exit 1; }
echo EXIT 0

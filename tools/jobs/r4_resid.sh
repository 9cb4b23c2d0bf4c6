# End-of-solve true-residual check: kResid vs a CPU rho, the recurrence gap by
# node class (tools/resid_probe.py), and pe_hip --json on the BASELINE grids
# (zero / random init, drift fault hook) -> profiles/r4_resid.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PROBE_GRID=${PGRID:-2048x2048,1000x1500} PROBE_INIT=zero,random timeout -k 10 300 python -u tools/resid_probe.py > $O/r4_resid_probe.txt 2>&1 || { tail -20 $O/r4_resid_probe.txt; exit 1; }
{
for g in ${GRIDS:-"2048 2048" "8192 8192"}; do
  for init in zero random; do
    echo "== $g init $init"; timeout -k 10 120 bin/pe_hip --json --quiet --init $init $g || exit 1
    echo "== $g init $init --algo fused"; timeout -k 10 120 bin/pe_hip --json --quiet --init $init --algo fused $g || exit 1
  done
done
echo "== 2048 drift@iter:900,amp:1e-3"
PE_FAULT_INJECT=drift@iter:900,amp:1e-3 timeout -k 10 120 bin/pe_hip --json --quiet 2048 2048 || exit 1
} > $O/r4_resid.txt 2>&1 || { tail -20 $O/r4_resid.txt; exit 1; }
echo EXIT 0

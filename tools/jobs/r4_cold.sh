# 400x600 T_solver as the FIRST process of a fresh box (round 3 measured 0.17-0.22 s
# there vs ~0.05 s later): construction-phase trace (PE_CTOR_TRACE=1) of the
# first and second process, then the HIP first-use probe -> profiles/r4_cold.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
{
for i in 1 2 3; do
  echo "== process $i: PE_CTOR_TRACE=1 bin/pe_hip --json 400 600"
  t0=$(date +%s.%N)
  PE_CTOR_TRACE=1 timeout -k 10 60 bin/pe_hip --json --quiet 400 600 2>&1 || exit 1
  echo "process wall $(python3 -c "print(round($(date +%s.%N) - $t0, 3))") s"
done
} > $O/r4_cold.txt 2>&1 || { tail -20 $O/r4_cold.txt; exit 1; }
echo EXIT 0

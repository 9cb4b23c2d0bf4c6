# Round 6, twenty-fifth GPU call: where the filling layout's host time goes
# (PE_CTOR_TRACE=3 laps per pass), one 8-rank slab construction.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twentyfifth; mkdir -p $O
cd $R
PE_CTOR_TRACE=3 PROBE_CFG=8:rows timeout -k 10 200 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -20 $O/ctor.txt; exit 1; }
grep -E "layout|re-layout|construction" $O/ctor.txt | head -150
echo EXIT 0

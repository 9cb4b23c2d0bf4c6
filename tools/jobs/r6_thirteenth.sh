# Round 6, thirteenth GPU call: where the halo-path choice's time goes
# (PE_CTOR_TRACE=2: reset, switch and timing per candidate), 8-rank slab.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirteenth; mkdir -p $O
cd $R
PROBE_CFG=8:rows PE_CTOR_TRACE=2 timeout -k 10 300 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -30 $O/ctor.txt; exit 1; }
grep -E "halo path|construction|ctor" $O/ctor.txt
echo EXIT 0

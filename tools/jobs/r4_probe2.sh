# Stamped timelines by layout (per-XCD / per-round uniform step cost, wave time vs
# static cost), DRAM counters per layout (8192^2 and one 8-rank 1024x8191 block
# on one GPU via --vranks? no: pe_hip 1024 8191 is a different problem, so the
# block is timed with tools/block_probe only), the three-step 2-D overlap probe
# (delay transport) -> profiles/r4_probe2.txt, profiles/r4_dram.txt, profiles/r4_overlap.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
{
PROBE_CFG=1:device PROBE_ENV="PE_LAYOUT=lpt;PE_LAYOUT=equal" timeout -k 10 300 python -u tools/stamp_probe.py || exit 1
PROBE_CFG=8:device PROBE_ENV="PE_LAYOUT=equal;PE_LAYOUT=lpt" timeout -k 10 300 python -u tools/stamp_probe.py || exit 1
} > $O/r4_probe2.txt 2>&1 || { tail -20 $O/r4_probe2.txt; exit 1; }
bash tools/jobs/r4_dram.sh > $O/r4_dram.txt 2>&1 || { tail -20 $O/r4_dram.txt; exit 1; }
PROBE_CFG=8:4x2,4:2x2 PROBE_OV=0,1:8 PROBE_GRAPH=0 timeout -k 10 300 python -u tools/overlap_probe.py 15 8 > $O/r4_overlap.txt 2>&1 || { tail -20 $O/r4_overlap.txt; exit 1; }
echo EXIT 0

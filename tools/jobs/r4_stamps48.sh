# Stamped kS3 timelines at the final configuration (aligned strips; 8192^2
# 112-row LPT items; the 8-rank slab block's tuned layout): per-item /
# per-wave timing, tail, per-step cost by kind -> profiles/r4_stamps48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PROBE_CFG=1:device,8:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/r4_stamps48.txt 2>&1 || { tail -20 $O/r4_stamps48.txt; exit 1; }
grep -v amdgpu.ids $O/r4_stamps48.txt | head -80
echo EXIT 0

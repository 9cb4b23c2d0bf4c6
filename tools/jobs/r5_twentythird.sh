# Round 5, twenty-third GPU call: the launch prologue broken down (state read
# and stop tests decided, step scalars formed, walk entered, first item) at the
# 8-rank slab, 2048^2 and 8192^2 (stamped build).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5twentythird; mkdir -p $O
cd $R
PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
PROBE_GRID=2048x2048 PROBE_CFG=1:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/stamps2048.txt 2>&1 || { tail -20 $O/stamps2048.txt; exit 1; }
grep -h -E "^P=|launch timeline|gap after|wave kernel entry|state read|step scalars|walk entry|first item start|last wave exit|last block|kernel entry \(wave\)|prologue issued|after row step 6 |after row step 12 " $O/stamps.txt $O/stamps2048.txt
echo EXIT 0

# Round 5, tenth GPU call: does a slow item stay slow when its list runs on
# another workgroup (PE_WPERM=1 reversed, 2 rotated by a quarter grid)?  Item
# speed by row / strip / workgroup decile at the 8-rank slab, 2048^2, 8192^2.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5tenth; mkdir -p $O
cd $R
PROBE_ENV="PE_WPERM=0;PE_WPERM=1;PE_WPERM=2" PROBE_CFG=8:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/slab.txt 2>&1 || { tail -20 $O/slab.txt; exit 1; }
PROBE_ENV="PE_WPERM=0;PE_WPERM=1;PE_WPERM=2" PROBE_GRID=2048x2048 PROBE_CFG=1:device timeout -k 10 200 python -u tools/stamp_probe.py > $O/g2048.txt 2>&1 || { tail -20 $O/g2048.txt; exit 1; }
PROBE_ENV="PE_WPERM=0;PE_WPERM=1" PROBE_CFG=1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/g8192.txt 2>&1 || { tail -20 $O/g8192.txt; exit 1; }
grep -h -E "^P=|by row decile|by workgroup decile|by strip decile|by XCD|tail \(|busy fraction" $O/slab.txt $O/g2048.txt $O/g8192.txt
echo EXIT 0

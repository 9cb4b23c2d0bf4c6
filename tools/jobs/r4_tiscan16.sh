# Rows per item at 16384^2 (aligned strips, LPT; layout_probe, two rounds at
# one placement) -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PROBE_GRID=16384x16384 PROBE_ITERS=120 PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="256;272;320;416;448;480;512" timeout -k 10 400 python -u tools/layout_probe.py > $O/r4_tiscan16.txt 2>&1 || { tail -20 $O/r4_tiscan16.txt; exit 1; }
cat $O/r4_tiscan16.txt
echo EXIT 0

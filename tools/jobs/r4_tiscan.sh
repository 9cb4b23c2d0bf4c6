# Rows-per-item scan of the LPT layout at 8192^2 and 16384^2 (aligned
# strips; tools/layout_probe.py, one placement per grid) -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
{
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="112;64;72;84;88;92;124;132;136;144;176;192;224" timeout -k 10 300 python -u tools/layout_probe.py || exit 1
PROBE_GRID=16384x16384 PROBE_ITERS=120 PROBE_P=1 PROBE_ROUNDS=1 PROBE_CFGS="256;224;240;272;288;320;384;448" timeout -k 10 300 python -u tools/layout_probe.py || exit 1
} > $O/r4_tiscan.txt 2>&1 || { tail -20 $O/r4_tiscan.txt; exit 1; }
cat $O/r4_tiscan.txt
echo EXIT 0

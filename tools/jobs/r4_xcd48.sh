# XCD-aware list placement (PE_XCD_MAP=1: neighbouring strips on one XCD's L2)
# with the aligned 48-column strips, one placement per block -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
{
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="112 PE_LAYOUT=lpt;112 PE_LAYOUT=lpt PE_XCD_MAP=1;80 PE_LAYOUT=lpt;80 PE_LAYOUT=lpt PE_XCD_MAP=1" timeout -k 10 240 python -u tools/layout_probe.py || exit 1
PROBE_P=8 PROBE_ROUNDS=2 PROBE_CFGS="80;80 PE_XCD_MAP=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
} > $O/r4_xcd48.txt 2>&1 || { tail -20 $O/r4_xcd48.txt; exit 1; }
cat $O/r4_xcd48.txt
echo EXIT 0

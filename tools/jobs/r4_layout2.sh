# Three-step equal-cost layout (exactly k equal-cost pieces per wave, PE_LAYOUT
# default) vs the filling (PE_LAYOUT=fill) and LPT (PE_LAYOUT=lpt) layouts and
# alternating march directions, at one placement per block (tools/layout_probe.py);
# stamped timeline of the equal layout -> profiles/r4_layout2.txt, profiles/r4_stamps_equal.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
{
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="80 PE_LAYOUT=lpt;80 PE_LAYOUT=lpt PE_ALTDIR=1;80;96;128;80 PE_ALTDIR=1;128 PE_ALTDIR=1" timeout -k 10 240 python -u tools/layout_probe.py || exit 1
PROBE_P=8 PROBE_ROUNDS=2 PROBE_CFGS="41 PE_LAYOUT=lpt;41;64;80;64 PE_ALTDIR=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_P=2 PROBE_ROUNDS=2 PROBE_CFGS="96 PE_LAYOUT=lpt;96 PE_LAYOUT=fill;96;80;64;128" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_P=4 PROBE_ROUNDS=2 PROBE_CFGS="64 PE_LAYOUT=lpt;64 PE_LAYOUT=fill;64;80;96" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
} > $O/r4_layout2.txt 2>&1 || { tail -20 $O/r4_layout2.txt; exit 1; }
PROBE_CFG=1:device,8:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/r4_stamps_equal.txt 2>&1 || { tail -20 $O/r4_stamps_equal.txt; exit 1; }
echo EXIT 0

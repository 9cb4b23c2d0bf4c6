# Three-step filling layout (kind-aware costs, items cut to fill every wave)
# vs the LPT layout, at one placement per block (tools/layout_probe.py), and
# the stamped timeline of the filling layout -> profiles/r4_layout.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
{
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="80 PE_LAYOUT=lpt;80;96;128;80 PE_ALTDIR=1;128 PE_ALTDIR=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_P=8 PROBE_ROUNDS=2 PROBE_CFGS="41 PE_LAYOUT=lpt;41;32;64;80;128;64 PE_ALTDIR=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_P=2 PROBE_ROUNDS=2 PROBE_CFGS="96 PE_LAYOUT=lpt;96;64;128;96 PE_ALTDIR=1" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_P=4 PROBE_ROUNDS=2 PROBE_CFGS="64 PE_LAYOUT=lpt;64;48;96" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
} > $O/r4_layout.txt 2>&1 || { tail -20 $O/r4_layout.txt; exit 1; }
PROBE_CFG=1:device,8:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/r4_stamps_fill.txt 2>&1 || { tail -20 $O/r4_stamps_fill.txt; exit 1; }
echo EXIT 0

# Do 112-row LPT items (the 8192^2 pick) help the tuned mid-size blocks?
# The 2-rank / 4-rank 8192^2 blocks and 4096^2 at one placement each
# (tools/layout_probe.py; first entry = the block's tuned default) -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
{
PROBE_P=2 PROBE_ROUNDS=2 PROBE_CFGS="88;112 PE_LAYOUT=lpt;112;132 PE_LAYOUT=lpt;96 PE_LAYOUT=lpt" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_P=4 PROBE_ROUNDS=2 PROBE_CFGS="90;112 PE_LAYOUT=lpt;112;132 PE_LAYOUT=lpt" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
PROBE_GRID=4096x4096 PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="64;112 PE_LAYOUT=lpt;112;132 PE_LAYOUT=lpt" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
} > $O/r4_mid112.txt 2>&1 || { tail -20 $O/r4_mid112.txt; exit 1; }
grep -v amdgpu.ids $O/r4_mid112.txt
echo EXIT 0

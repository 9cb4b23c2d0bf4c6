# Rows per item of the big single-rank blocks, aligned 48-column strips, a
# second box (tools/layout_probe.py at one placement per block) -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
{
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="80 PE_LAYOUT=lpt;104 PE_LAYOUT=lpt;112 PE_LAYOUT=lpt;120 PE_LAYOUT=lpt;160 PE_LAYOUT=lpt" timeout -k 10 240 python -u tools/layout_probe.py || exit 1
PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="112 PE_LAYOUT=lpt;128 PE_LAYOUT=lpt;160 PE_LAYOUT=lpt;192 PE_LAYOUT=lpt;256 PE_LAYOUT=lpt" timeout -k 10 300 python -u tools/layout_probe.py || exit 1
PROBE_GRID=4096x4096 PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="64;80;96;112" timeout -k 10 200 python -u tools/layout_probe.py || exit 1
} > $O/r4_ti48b.txt 2>&1 || { tail -20 $O/r4_ti48b.txt; exit 1; }
cat $O/r4_ti48b.txt
echo EXIT 0

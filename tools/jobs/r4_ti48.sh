# Rows per item and layout for the big blocks with the aligned 48-column
# strips (tools/layout_probe.py at one placement: 8192^2 and 16384^2), then
# the driver-shaped / long bench -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
{
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="80 PE_LAYOUT=lpt;96 PE_LAYOUT=lpt;112 PE_LAYOUT=lpt;128 PE_LAYOUT=lpt;96 PE_LAYOUT=fill;96 PE_LAYOUT=equal" timeout -k 10 240 python -u tools/layout_probe.py || exit 1
PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="80 PE_LAYOUT=lpt;96 PE_LAYOUT=lpt;128 PE_LAYOUT=lpt" timeout -k 10 300 python -u tools/layout_probe.py || exit 1
} > $O/r4_ti48.txt 2>&1 || { tail -20 $O/r4_ti48.txt; exit 1; }
cat $O/r4_ti48.txt
timeout -k 10 180 python -u bench.py --steps 20 --warmup 5 > $O/r4_ti48_b20.json 2> $O/r4_ti48_b20.err || { tail $O/r4_ti48_b20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/r4_ti48_b20.json')); print('bench20', d['value'], d['ms_per_step'], d['config']['rows_per_item'])"
timeout -k 10 180 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/r4_ti48_b2000.json 2> $O/r4_ti48_b2000.err || { tail $O/r4_ti48_b2000.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/r4_ti48_b2000.json')); print('bench2000', d['value'], d['ms_per_step'], d['config']['placement'])"
echo EXIT 0

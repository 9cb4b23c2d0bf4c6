# Round 5, forty-third GPU call: the exchange path's per-rank time at 15 / 8 us
# delays for the 2-rank slab of 8192^2 and the 8-rank slab of 16384^2 (the
# projection rows the default halo path had not been timed for).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5fortythird; mkdir -p $O
cd $R
PROBE_CFG=2:device PROBE_GRAPH=0 timeout -k 10 300 python -u tools/overlap_probe.py 15 8 > $O/ov8192.txt 2>&1 || { tail -20 $O/ov8192.txt; exit 1; }
grep -h "us/iter" $O/ov8192.txt
PROBE_GRID=16384x16384 PROBE_CFG=8:device PROBE_GRAPH=0 timeout -k 10 300 python -u tools/overlap_probe.py 15 8 > $O/ov16k.txt 2>&1 || { tail -20 $O/ov16k.txt; exit 1; }
grep -h "us/iter" $O/ov16k.txt
echo EXIT 0

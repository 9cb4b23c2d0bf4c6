# Round 6, seventh GPU call: short vs steady timing of the overlap (the
# construction's 4-sweep candidates vs 300-iteration windows), 8-rank slab
# and 4x2 block of 8192^2.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6seventh; mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/overlap_steady_probe.py > $O/steady.txt 2>&1 || { tail -20 $O/steady.txt; exit 1; }
PROBE_SPEC=4x2 PROBE_LOOP=1 timeout -k 10 300 python -u tools/overlap_steady_probe.py >> $O/steady.txt 2>&1 || { tail -20 $O/steady.txt; exit 1; }
cat $O/steady.txt
echo EXIT 0

# Round 6, thirty-ninth GPU call: does memory placement matter for the
# multi-rank blocks (no placement search below 24 M nodes)?  Fresh solvers of
# the 8- and 4-rank slab blocks of 8192² with the search forced (12 tries,
# every candidate's ms per sweep) and without it (1 try), 300 iterations each.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirtyninth; mkdir -p $O
cd $R
PE_PLACEMENT_TRIES=12 PROBE_REPS=3 timeout -k 10 300 python -u tools/placement_probe.py > $O/p12.txt 2>&1 || { tail -20 $O/p12.txt; exit 1; }
grep "^P=" $O/p12.txt
PE_PLACEMENT_TRIES=1 PROBE_REPS=4 timeout -k 10 300 python -u tools/placement_probe.py > $O/p1.txt 2>&1 || { tail -20 $O/p1.txt; exit 1; }
grep "^P=" $O/p1.txt
echo EXIT 0

# Round 6, forty-first GPU call: a best-of-8 placement (12 GB spacers) for multi-GPU mid-size
# blocks (forced on the delay transport with PE_PLACEMENT_TRIES=8: no stop
# rule, no retry round), fresh solvers of the 8- and 4-rank slab blocks; the
# (measured, not adopted)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6forty-first; mkdir -p $O
cd $R
PE_PLACEMENT_TRIES=8 PROBE_REPS=4 timeout -k 10 300 python -u tools/placement_probe.py > $O/p8.txt 2>&1 || { tail -20 $O/p8.txt; exit 1; }
grep "^P=" $O/p8.txt
echo EXIT 0

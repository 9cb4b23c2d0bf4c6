# Round 6, fortieth GPU call: the best-of-4 placement for multi-GPU mid-size
# blocks (forced on the delay transport with PE_PLACEMENT_TRIES=4: no stop
# rule, no retry round), fresh solvers of the 8- and 4-rank slab blocks; the
# multi-process GPU tests (the search was not adopted).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fortieth; mkdir -p $O
cd $R
PE_PLACEMENT_TRIES=4 PROBE_REPS=3 timeout -k 10 300 python -u tools/placement_probe.py > $O/p4.txt 2>&1 || { tail -20 $O/p4.txt; exit 1; }
grep "^P=" $O/p4.txt
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py -m gpu -k "agrees or multi_process or bench" > $O/t.txt 2>&1 || { tail -40 $O/t.txt; exit 1; }
tail -1 $O/t.txt
echo EXIT 0

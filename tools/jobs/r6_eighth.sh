# Round 6, eighth GPU call: the construction's short timing of each halo arm
# against its 300-iteration steady state, on one solver (set_halo_path).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6eighth; mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/overlap_steady_probe.py > $O/steady.txt 2>&1 || { tail -20 $O/steady.txt; exit 1; }
cat $O/steady.txt
echo EXIT 0

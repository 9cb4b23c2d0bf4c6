# Round 6, forty-sixth GPU call: the placement search on the 2-rank block of
# 8192² (33.5 M nodes: searched, but the 8192²-calibrated stop rate is never
# reached there) — one fresh process per construction, candidates and search
# time.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fortysixth; mkdir -p $O
cd $R
for i in 1 2 3; do
  PE_PLACEMENT_TRIES=12 PROBE_CFG=2:rows PROBE_REPS=1 timeout -k 10 200 python -u tools/placement_probe.py > $O/p_$i.txt 2>&1 || { tail -20 $O/p_$i.txt; exit 1; }
  grep "^P=" $O/p_$i.txt | cut -c1-400
done
echo EXIT 0

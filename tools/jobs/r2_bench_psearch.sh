# Placement search before (PE_PLACEMENT_LISTED=0) vs after the item layout (=1, now the default), static 8192^2 layout, alternating fresh processes -> profiles/r2_bench_psearch.txt
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  PE_PLACEMENT_LISTED=0 timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1
  PE_PLACEMENT_LISTED=1 timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1
done

# Headline bench with the tail split off (new default) vs on (PE_TAIL_FRAC=0.3), alternating fresh processes.
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1
  PE_TAIL_FRAC=0.3 timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1
done

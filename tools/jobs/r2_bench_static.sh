# Headline bench: static LPT layout with 24-row items (PE_ORDER=0 PE_TI=24) vs the dynamic queue (default), alternating fresh processes; 16384^2 layouts at one placement.
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  PE_ORDER=0 PE_TI=24 timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1
  timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1
done
PROBE_GRID=16384x16384 PROBE_P=1 PROBE_ITERS=100 PROBE_CFGS="18d;24s;30s;18d" timeout -k 10 200 python3 -u tools/layout_probe.py 2>&1 | grep -v amdgpu.ids || exit 1

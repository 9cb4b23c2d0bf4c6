# Static layouts with taller items at one placement: 4096^2 (tuned among 8-18 today), the 2-rank 8192^2 block (24 fixed), 2400x3200.
cd $GRAFT_REPO_ROOT
probe() { timeout -k 10 200 python3 -u tools/layout_probe.py 2>&1 | grep -v amdgpu.ids; }
PROBE_GRID=4096x4096 PROBE_CFGS="14s;18s;24s;30s;36s" probe || exit 1
PROBE_P=2 PROBE_CFGS="24s;30s;36s;20s" probe || exit 1
PROBE_GRID=2400x3200 PROBE_CFGS="11s;18s;24s;30s" probe || exit 1
PROBE_GRID=1600x2400 PROBE_CFGS="10s;18s;24s" probe || exit 1

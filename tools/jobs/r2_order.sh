# Static LPT layout vs dynamic queue at ONE placement per block (tools/layout_probe.py, relayout with an order): 1-, 2-, 4-rank blocks of 8192^2 -> profiles/r2_order.txt
cd $GRAFT_REPO_ROOT
probe() { timeout -k 10 250 python3 -u tools/layout_probe.py 2>&1 | grep -v amdgpu.ids; }
PROBE_P=1 PROBE_CFGS="18d;18s;24s;30s;36s;22d" probe || exit 1
PROBE_P=2 PROBE_CFGS="18d;18s;24s;30s;36s;22d" probe || exit 1
PROBE_P=4 PROBE_CFGS="23s;18d;16s;24s;30s" probe || exit 1

# Big blocks (8192^2 on 1 rank, the 2-rank block, 4096^2): dynamic queue (default) vs the static LPT layout (tuned / fixed item heights).
cd $GRAFT_REPO_ROOT
E=" ;PE_ORDER=0;PE_ORDER=0 PE_TI=18;PE_ORDER=0 PE_TI=30; "
PROBE_CFG=1:device,2:device PROBE_ENV="$E" timeout -k 10 300 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_GRID=4096x4096 PROBE_CFG=1:device PROBE_ENV="$E" timeout -k 10 200 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1

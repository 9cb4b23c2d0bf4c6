# Mid blocks (4- and 8-rank 8192^2 blocks, 2400x3200): static tuned layout vs the dynamic queue without the tail split, several item heights.
cd $GRAFT_REPO_ROOT
E=" ;PE_ORDER=3 PE_TI=12;PE_ORDER=3 PE_TI=18;PE_ORDER=3 PE_TI=24;PE_ORDER=3 PE_TI=32; "
PROBE_CFG=8:device,4:device PROBE_ENV="$E" timeout -k 10 200 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_GRID=2400x3200 PROBE_CFG=1:device PROBE_ENV="$E" timeout -k 10 200 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1

# Static LPT layout: measured sweep time vs the layout's predicted wave load across item heights (4- and 8-rank blocks of 8192^2, 2400x3200).
cd $GRAFT_REPO_ROOT
C="8;9;10;11;12;13;14;15;16;17;18;19;20;21;22;23;24;26;28"
PROBE_GRID=8192x8192 PROBE_P=4 PROBE_ROUNDS=1 PROBE_CFGS="$C" timeout -k 10 150 python3 -u tools/layout_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_GRID=8192x8192 PROBE_P=8 PROBE_ROUNDS=1 PROBE_CFGS="$C" timeout -k 10 150 python3 -u tools/layout_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_GRID=2400x3200 PROBE_P=1 PROBE_ROUNDS=1 PROBE_CFGS="$C" timeout -k 10 150 python3 -u tools/layout_probe.py 2>&1 | grep -v amdgpu.ids || exit 1

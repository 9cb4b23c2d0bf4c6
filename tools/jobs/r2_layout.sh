# Item-layout knobs at one memory placement (tools/layout_probe.py) -> profiles/r2_layout.txt.
# Runs 1-3: the dynamic queue's tail split / item height at 1, 2 and 4 ranks of 8192^2 (the 4-rank block is static);
# run 4: static LPT layouts, measured vs predicted wave load across item heights.
cd $GRAFT_REPO_ROOT
probe() { timeout -k 10 200 python3 -u tools/layout_probe.py 2>&1 | grep -v amdgpu.ids; }
PROBE_P=1 PROBE_CFGS="18;18 PE_TAIL_FRAC=0.3;18 PE_TAIL_FRAC=0.3 PE_TAIL_SPLIT=3;18 PE_TAIL_FRAC=0.1;18 PE_TAIL_FRAC=0.05;22;26;18 PE_HEAVY_FIRST=0;18 PE_GEN_COST=2" probe || exit 1
for P in 2 4; do PROBE_P=$P PROBE_CFGS="18;18 PE_TAIL_FRAC=0.3;16;20;22;26" probe || exit 1; done
PROBE_P=8 PROBE_CFGS="10;12;12 PE_GEN_COST=2;12 PE_GEN_COST=1.5;12 PE_HEAVY_SPLIT=0" probe || exit 1
C="8;9;10;11;12;13;14;15;16;17;18;19;20;21;22;23;24;26;28"
for P in 4 8; do PROBE_P=$P PROBE_ROUNDS=1 PROBE_CFGS="$C" probe || exit 1; done
PROBE_GRID=2400x3200 PROBE_P=1 PROBE_ROUNDS=1 PROBE_CFGS="$C" probe || exit 1

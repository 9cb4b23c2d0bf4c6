# Round 2: ~8 M-node blocks (2400x3200 on one GPU; one rank's 1024x8191 block of an
# 8-rank 8192^2 run): item order (static LPT / dynamic per-XCD queue) x rows per item x stores.
set -o pipefail
cd $GRAFT_REPO_ROOT
ENVS="PE_ORDER=0 PE_TI=10;PE_ORDER=0 PE_TI=14;PE_ORDER=0 PE_TI=18;PE_ORDER=3 PE_TI=8;PE_ORDER=3 PE_TI=10;PE_ORDER=3 PE_TI=14;PE_ORDER=3 PE_TI=18;PE_ORDER=3 PE_TI=14 PE_SKERNEL=1;PE_ORDER=0 PE_TI=10 PE_SKERNEL=1"
PROBE_CFG=8:device PROBE_ENV="$ENVS" timeout -k 10 300 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_GRID=2400x3200 PROBE_CFG=1:aspect PROBE_ENV="$ENVS" timeout -k 10 300 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
PROBE_GRID=1600x2400 PROBE_CFG=1:aspect PROBE_ENV="$ENVS" timeout -k 10 300 python3 -u tools/block_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
echo EXIT 0

set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/orders; mkdir -p $O
timeout -k 10 400 python tools/cfg_probe.py PE_ORDER=3 PE_ORDER=0 PE_ORDER=2 PE_ORDER=3,PE_TI=8 PE_ORDER=3,PE_TI=32 PE_ORDER=3 PE_ORDER=0 > $O/cfg.txt 2>&1 || { tail $O/cfg.txt; exit 1; }
PROBE_GRID=2900 timeout -k 10 400 python tools/cfg_probe.py PE_ORDER=3 PE_ORDER=0 PE_ORDER=3,PE_TI=8 PE_ORDER=0,PE_TI=8 >> $O/cfg.txt 2>&1 || { tail $O/cfg.txt; exit 1; }
grep -v amdgpu.ids $O/cfg.txt

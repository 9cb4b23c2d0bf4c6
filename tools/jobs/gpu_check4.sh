set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/check4; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 400 python tools/cfg_probe.py PE_ORDER=3 PE_ORDER=0 PE_ORDER=3 PE_ORDER=3,PE_TI=24 > $O/cfg.txt 2>&1 || { tail $O/cfg.txt; exit 1; }
PROBE_GRID=2900 timeout -k 10 400 python tools/cfg_probe.py PE_ORDER=0 PE_ORDER=3 PE_ORDER=0,PE_TI=16 >> $O/cfg.txt 2>&1 || { tail $O/cfg.txt; exit 1; }
grep -v amdgpu.ids $O/cfg.txt

# GPU tests + 8192² configuration probe (same process, several allocations).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/check2; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python tools/cfg_probe.py PE_TI=16 PE_TI=8 PE_TI=16,PE_SKERNEL=2 PE_TI=16,PE_SKERNEL=3 PE_TI=16 PE_TI=16 > $O/cfg.txt 2>&1 || { tail $O/cfg.txt; exit 1; }
grep -v amdgpu.ids $O/cfg.txt
timeout -k 10 100 bin/pe_hip --json --quiet 8192 8192 | cut -c1-200

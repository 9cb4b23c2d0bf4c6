# Aligned three-step strips (48 outputs of 64 lanes, rows' element 0 at column
# -7: whole 128-B line loads, whole 64-B segment stores): three-step / layout /
# residual GPU tests, the dynamic sweep's single-sweep check, per-block speed
# (tools/layout_probe.py) and 8192^2 DRAM counters -> profiles/r4_align.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --tb=short --timeout 200 --timeout-method thread tests/test_three_step.py tests/test_layout.py tests/test_residual.py > $O/r4_align_tests.txt 2>&1 || { tail -30 $O/r4_align_tests.txt; exit 1; }
tail -2 $O/r4_align_tests.txt
PE_DYN3=1 timeout -k 10 200 python -u -m pytest -x -q --tb=short --timeout 100 --timeout-method thread tests/test_three_step.py > $O/r4_align_dyn.txt 2>&1; echo "dyn tests rc=$?"; tail -4 $O/r4_align_dyn.txt
{
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="80 PE_LAYOUT=lpt;96 PE_LAYOUT=lpt;64 PE_LAYOUT=lpt;80 PE_LAYOUT=lpt PE_DYN3=1" timeout -k 10 240 python -u tools/layout_probe.py || exit 1
PROBE_CFG=8:device,4:device,2:device,8:4x2 timeout -k 10 300 python3 -u tools/block_probe.py || exit 1
} > $O/r4_align.txt 2>&1 || { tail -20 $O/r4_align.txt; exit 1; }
cat $O/r4_align.txt
CFGS="PE_LAYOUT=lpt" bash tools/jobs/r4_dram.sh > $O/r4_align_dram.txt 2>&1 || { tail -20 $O/r4_align_dram.txt; exit 1; }
cat $O/r4_align_dram.txt
PE_CTOR_TRACE=1 timeout -k 10 100 bin/pe_hip --json --quiet 16384 16384 > $O/r4_ctor16k.txt 2>&1 || { tail -20 $O/r4_ctor16k.txt; exit 1; }
tail -30 $O/r4_ctor16k.txt
echo EXIT 0

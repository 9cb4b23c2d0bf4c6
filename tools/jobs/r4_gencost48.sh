# Band-row cost weight of the LPT layout at 8192^2 with 112-row items
# (PE_GEN_COST; default 3), one placement (tools/layout_probe.py) -> profiles/r4_ti48.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PROBE_P=1 PROBE_ROUNDS=2 PROBE_CFGS="${CFGS:-112;112 PE_GEN_COST=2;112 PE_GEN_COST=2.25;112 PE_GEN_COST=2.5;112 PE_GEN_COST=3.5;112 PE_HEAVY_SPLIT=0}" timeout -k 10 240 python -u tools/layout_probe.py > $O/r4_gencost48.txt 2>&1 || { tail -20 $O/r4_gencost48.txt; exit 1; }
grep -v amdgpu.ids $O/r4_gencost48.txt
echo EXIT 0

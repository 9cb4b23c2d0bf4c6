# Per-item timeline of the three-step sweep (PE_STAMPS=1 build of kS3):
# item durations by kind (uniform / mixed / band) and per-wave load balance,
# 8192^2 on 1 GPU and the 8-rank row-slab block -> profiles/r4_stamps.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
PROBE_CFG=1:device,8:device,2:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/r4_stamps.txt 2>&1 <<< "" || { tail -20 $O/r4_stamps.txt; exit 1; }
timeout -k 10 200 python -u bench.py --steps 600 --warmup 20 > $O/r4_bench600.txt 2>&1 || { tail -20 $O/r4_bench600.txt; exit 1; }
echo EXIT 0

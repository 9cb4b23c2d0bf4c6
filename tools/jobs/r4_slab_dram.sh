# DRAM request counters of the 8-rank slab block's sweep (8 virtual ranks of
# 8192^2 on one GPU, row slabs 1024x8191: one kS3 dispatch per rank and
# sweep), TCC_EA0_RDREQ (x128 B) / WRREQ (x64 B) -> profiles/r4_slab_dram.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4slab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/p -o run -- $R/bin/pe_hip --quiet --vranks 8 --max-iter 150 --no-tol 8192 8192 > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
cd $R
db=$(ls $O/p/run_results.db $O/p/*/run_results.db 2>/dev/null | tail -1)
python3 tools/pmc_by_dispatch.py $db --kernel kS3 --by-name
echo EXIT 0

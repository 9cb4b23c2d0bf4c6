# Final-config profiles (aligned strips, 112-row items) at 8192^2: TCC_EA0
# DRAM request counters per kS3 dispatch at the default and at 80 rows
# (tools/jobs/r4_dram.sh), then a kernel trace + stats of the driver-shaped
# bench (its last timed window) -> profiles/r4_prof.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4prof; mkdir -p $O
cd $R
CFGS="PE_LAYOUT=lpt PE_TI=80" bash tools/jobs/r4_dram.sh > $O/dram.txt 2>&1 || { tail -20 $O/dram.txt; exit 1; }
cat $O/dram.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-solve > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
cd $R
db=$(ls $O/kt/run_results.db $O/kt/*/run_results.db 2>/dev/null | tail -1)
python3 tools/rocpd_summary.py $db --timeline 12 > $O/kt.txt 2>&1 || { tail $O/kt.txt; exit 1; }
cat $O/kt.txt | head -40
grep '^{' $O/kt.log | tail -1 | cut -c1-300
echo EXIT 0

# Round 5, first GPU call: (1) DRAM counter calibration on kernels of known
# byte counts (tools/micro/counter_cal.hip) -> profiles/r5_counter_calibration.txt;
# (2) per-rank block probes at HEAD for every BASELINE config and the
# reference's 2-GPU grids -> profiles/r5_block_probe_base.txt; (3) s = 4
# moment-form numerics (golden counts, scalar drift, recurrence gap) ->
# profiles/r5_sstep4.txt
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5first; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pass in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_64B_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  tag=$(echo $pass | tr ' ' '+')
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pass -d $O/cal_$tag -o run -- $R/bin/counter_cal > $O/cal_$tag.log 2>&1
  echo "pass [$pass] rc $?"
done
cd $R
for d in $O/cal_*; do
  [ -d $d ] || continue
  db=$(ls $d/run_results.db $d/*/run_results.db 2>/dev/null | tail -1)
  [ -n "$db" ] && { echo "== $d"; python3 tools/pmc_by_dispatch.py $db --kernel k --by-name --skip 0; }
done > $O/cal_summary.txt 2>&1
cat $O/cal_summary.txt
grep -h "rep 2\|geometry" $O/cal_TCC_EA0_RDREQ_sum+TCC_EA0_WRREQ_sum.log
PROBE_CFG=2:device,4:device,8:device,8:4x2 timeout -k 10 240 python -u tools/block_probe.py > $O/probe8192.txt 2>&1; echo "probe8192 rc $?"
PROBE_GRID=16384x16384 PROBE_ITERS=150 PROBE_CFG=2:device,4:device,8:device timeout -k 10 240 python -u tools/block_probe.py > $O/probe16384.txt 2>&1; echo "probe16384 rc $?"
PROBE_GRID=4096x4096 PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe4096.txt 2>&1; echo "probe4096 rc $?"
for g in 800x1200 1600x2400 2400x3200 2048x2048; do
  PROBE_GRID=$g PROBE_CFG=2:device timeout -k 10 120 python -u tools/block_probe.py > $O/probe$g.txt 2>&1; echo "probe$g rc $?"
done
grep -h "us/iter" $O/probe*.txt
timeout -k 10 600 python -u tools/sstep_proto.py 4 cuda 800x1200 1600x2400 2400x3200 2048x2048 4096x4096 2048x2048r 8192x8192 > $O/sstep4.txt 2>&1; echo "sstep4 rc $?"
timeout -k 10 300 python -u tools/sstep_proto.py 3 cuda 2048x2048 2048x2048r 8192x8192 > $O/sstep3.txt 2>&1; echo "sstep3 rc $?"
grep -h "^s=" $O/sstep4.txt $O/sstep3.txt
echo EXIT 0

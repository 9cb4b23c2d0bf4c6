# Issue / VALU / memory-instruction counters of the two sweep variants (applying WM=2, deferring WM=0): 8192^2 (dynamic) and the 8-rank block (static) -> profiles/r2_sweep_pmc.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/spmc; mkdir -p $O
export PROBE_ITERS=120
for cfg in 1:device 8:device; do
  n=${cfg%%:*}
  PROBE_CFG=$cfg timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY -d $O/a$n -o run -- python3 $R/tools/block_probe.py > $O/a$n.log 2>&1 || exit 1
  PROBE_CFG=$cfg timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/b$n -o run -- python3 $R/tools/block_probe.py > $O/b$n.log 2>&1 || exit 1
done
for f in $O/a1 $O/b1 $O/a8 $O/b8; do echo "== $f"; python3 $R/tools/pmc_by_dispatch.py $(ls $f/run_results.db $f/*/run_results.db 2>/dev/null | tail -1) --kernel kS --by-name || exit 1; done

# Quad layout (PE_QUAD=1: a workgroup's 4 waves take 4 adjacent strips of the
# same rows) vs the LPT layout, three-step sweep, at one memory placement per
# block (tools/layout_probe.py), then DRAM request counters of kS3 for both.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/quad; mkdir -p $O
cd $R
echo "== 8192^2, 1 rank"
PROBE_GRID=8192x8192 PROBE_P=1 PROBE_ITERS=600 PROBE_ROUNDS=3 PROBE_CFGS="80;80 PE_QUAD=1;96 PE_QUAD=1;64 PE_QUAD=1" \
  timeout -k 10 200 python3 -u tools/layout_probe.py || exit 1
echo "== 8192^2 8-rank slab block"
PROBE_GRID=8192x8192 PROBE_P=8 PROBE_SPEC=rows PROBE_ITERS=600 PROBE_ROUNDS=2 PROBE_CFGS="32;32 PE_QUAD=1;64;86;103;128;86 PE_QUAD=1;103 PE_QUAD=1" \
  timeout -k 10 200 python3 -u tools/layout_probe.py || exit 1
echo "== 8192^2 2-rank slab block"
PROBE_GRID=8192x8192 PROBE_P=2 PROBE_SPEC=rows PROBE_ITERS=300 PROBE_ROUNDS=2 PROBE_CFGS="64;64 PE_QUAD=1" \
  timeout -k 10 200 python3 -u tools/layout_probe.py || exit 1
cd /tmp && export TMPDIR=/tmp
ARGS="--quiet --max-iter 300 --no-tol 8192 8192"
for q in 0 1; do
  PE_QUAD=$q timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/q$q -o run -- $R/bin/pe_hip $ARGS > $O/q$q.log 2>&1 || { tail $O/q$q.log; exit 1; }
done
cd $R
for q in 0 1; do
  db=$(ls $O/q$q/run_results.db $O/q$q/*/run_results.db 2>/dev/null | tail -1)
  echo "== PE_QUAD=$q counters"; python3 tools/pmc_by_dispatch.py $db --kernel kS3 --by-name || exit 1
done
echo EXIT 0

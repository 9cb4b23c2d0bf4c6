# Round 2: in-sweep halo push over xGMI (row slabs + in-sweep P2P sums) —
# multi-process tests on the one GPU (IPC-mapped receive buffers), bench with
# graph-captured multi-rank iterations, and the 1-GPU headline unchanged.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/push; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "halo_push or multi_process_2d" > $O/pytest.txt 2>&1; rc=$?
tail -15 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-solve > $O/bench1.json 2> $O/bench1.err || exit 1
cat $O/bench1.json
echo EXIT 0

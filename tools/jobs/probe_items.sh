# Item-queue variants: real sweep timings per rank block, stamps, the GPU tests, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/items; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
PROBE_CFG=8:aspect,8:rows,4:aspect,2:aspect PROBE_ITERS=300 \
PROBE_ENV="PE_ORDER=0;PE_ORDER=3 PE_TI=16 PE_TAIL_FRAC=0;PE_ORDER=3 PE_TI=16;PE_ORDER=3 PE_TI=16 PE_TAIL_FRAC=0.5;PE_ORDER=3 PE_TI=16 PE_TAIL_SPLIT=4;PE_ORDER=3 PE_TI=24 PE_TAIL_SPLIT=3;PE_ORDER=3 PE_TI=8" \
  timeout -k 10 500 python3 tools/block_probe.py > $O/block.txt 2>&1 || exit 1
PROBE_CFG=1:aspect PROBE_ITERS=300 \
PROBE_ENV="PE_TAIL_FRAC=0;PE_TAIL_FRAC=0.3;PE_TAIL_FRAC=0;PE_TAIL_FRAC=0.3;PE_TAIL_SPLIT=4;PE_TI=24 PE_TAIL_SPLIT=3" \
  timeout -k 10 300 python3 tools/block_probe.py >> $O/block.txt 2>&1 || exit 1
PROBE_CFG=8:aspect,1:aspect PROBE_ENV="PE_ORDER=3 PE_TI=16" timeout -k 10 200 python3 tools/stamp_probe.py > $O/stamps.txt 2>&1

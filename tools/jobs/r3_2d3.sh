# Three-step sweep on 2-D splits (exchange path): the multi-process tests on
# one GPU, the three-step suite; then one rank's 2-D block timed single sweep
# vs three-step (tools/block_probe.py); then the short-window probe.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3_2d3; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_three_step.py -m gpu -q -x --timeout 300 --timeout-method thread \
  -k "multi_process_2d or three_step" > $O/pytest.txt 2>&1; rc=$?
tail -15 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
PROBE_CFG=8:4x2,4:2x2,8:rows PROBE_ENV="PE_STEPS=1;PE_STEPS=3" timeout -k 10 300 python3 -u tools/block_probe.py || exit 1
timeout -k 10 150 python3 -u tools/window_probe.py || exit 1
echo EXIT 0

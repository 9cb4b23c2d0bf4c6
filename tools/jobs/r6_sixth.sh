# Round 6, sixth GPU call: the whole GPU suite (verbose: per-test progress),
# then the halo probe at the 8-rank splits (put with 8 blocks per message
# under the overlap).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6sixth; mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
PROBE_CFG=8:rows,8:4x2 PROBE_EACH=1 PROBE_ITERS=300 timeout -k 10 300 python -u tools/halo_probe.py 0 0 > $O/halo_probe.txt 2>&1 || { tail -20 $O/halo_probe.txt; exit 1; }
cat $O/halo_probe.txt
echo EXIT 0

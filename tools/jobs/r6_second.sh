# Round 6, second GPU call: the new halo paths (peer put, construction-time
# choice) — their tests first, then the whole GPU suite, then the 1-GPU bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6second; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu.py \
  -k "loopback_transport_bitwise or halo_path_choice or halo_put or host_staged or halo_push_graphs" > $O/new_tests.txt 2>&1 || { tail -40 $O/new_tests.txt; exit 1; }
grep -E "passed|failed" $O/new_tests.txt | tail -3
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
tail -1 $O/bench.txt | cut -c1-300
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
echo EXIT 0

# After making big blocks (<= 2^26 nodes) static: headline bench twice + the large golden solves.
cd $GRAFT_REPO_ROOT
for i in 1 2; do timeout -k 10 150 python3 bench.py --steps 400 --warmup 20 2>/dev/null | tail -1 || exit 1; done
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "large_golden or bench" 2>&1 | grep -E "PASS|FAIL|ERROR|passed|failed|assert" | tail -20

# Round 6, thirty-third GPU call: kernel traces of fresh solvers with the
# peer put's overlap forced (loopback put, the 8-rank slab), and the halo /
# overlap / layout GPU tests after the fallback change.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirtythird; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PROBE_HALO=put timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ovput -o run -- python3 $R/tools/overlap_trace_probe.py > $O/ovput.log 2>&1 || { tail -20 $O/ovput.log; exit 1; }
grep "^rep" $O/ovput.log | cut -c1-120
cd $R
db=$(ls $O/ovput/run_results.db $O/ovput/*/run_results.db 2>/dev/null | tail -1)
python3 tools/rocpd_summary.py $db --segments 5 > $O/ovput.summary.txt 2>&1
grep -E "segment|kS3|kWaitSig|kPut" $O/ovput.summary.txt | head -24
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_layout.py tests/test_gpu.py -m gpu -k "layout or tun or halo_path or overlap or resume or put" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
echo EXIT 0

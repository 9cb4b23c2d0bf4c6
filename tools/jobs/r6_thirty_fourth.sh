# Round 6, thirty-fourth GPU call: the halo choice builds the overlap's
# layouts ahead, on the host, under the GPU timing of the candidates before
# them — construction trace, layout / halo / overlap GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6thirtyfourth; mkdir -p $O
cd $R
PE_CTOR_TRACE=2 timeout -k 10 200 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -20 $O/ctor.txt; exit 1; }
grep -E "halo path (reset|re-layout|layout ahead|.*apply)|construction" $O/ctor.txt > $O/ctor_short.txt; grep construction $O/ctor_short.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_layout.py tests/test_gpu.py -m gpu -k "layout or tun or halo_path or overlap or resume or put" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
PROBE_REPS=3 timeout -k 10 200 python -u tools/overlap_trace_probe.py > $O/ov.txt 2>&1 || { tail -20 $O/ov.txt; exit 1; }
grep "^rep" $O/ov.txt | cut -c1-100
echo EXIT 0

# Round 6, eighteenth GPU call: the overlap timed at the rows-per-item
# tuning's two best heights — the variance probe, the construction cost, the
# halo-path tests and the projections.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6eighteenth; mkdir -p $O
cd $R
PROBE_REPS=6 timeout -k 10 300 python -u tools/overlap_trace_probe.py > $O/ov.txt 2>&1 || { tail -20 $O/ov.txt; exit 1; }
grep "^rep" $O/ov.txt
PE_CTOR_TRACE=2 timeout -k 10 200 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -20 $O/ctor.txt; exit 1; }
grep -v "^\[pe\] halo path" $O/ctor.txt | tail -12
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py -m gpu \
  -k "halo_path_choice or overlap_async_loopback or halo_put" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -2 $O/t.txt
PROBE_HALO=exchange timeout -k 10 400 python -u tools/halo_probe.py 0 0 15 8 > $O/proj.txt 2>&1 || { tail -20 $O/proj.txt; exit 1; }
cat $O/proj.txt
echo EXIT 0

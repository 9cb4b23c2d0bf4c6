# Round 6, twenty-first GPU call: the filling layout builds its per-wave
# lists once; the construction's layout seeds the choice's cache.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6twentyfirst; mkdir -p $O
cd $R
PROBE_REPS=6 timeout -k 10 300 python -u tools/overlap_trace_probe.py > $O/ov.txt 2>&1 || { tail -20 $O/ov.txt; exit 1; }
grep "^rep" $O/ov.txt
PE_CTOR_TRACE=3 timeout -k 10 200 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -20 $O/ctor.txt; exit 1; }
grep -E "halo path (reset|re-layout|.*apply)|construction" $O/ctor.txt > $O/ctor_short.txt; head -60 $O/ctor_short.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py -m gpu \
  -k "halo_path_choice or overlap_async_loopback or halo_put" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -2 $O/t.txt
PROBE_HALO=exchange timeout -k 10 400 python -u tools/halo_probe.py 0 0 15 8 > $O/proj.txt 2>&1 || { tail -20 $O/proj.txt; exit 1; }
cat $O/proj.txt
echo EXIT 0

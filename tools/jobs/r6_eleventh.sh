# Round 6, eleventh GPU call: the diagnostic-knob test, the construction cost
# of the halo-path choice (PE_CTOR_TRACE), a 4-process bench on the default
# path (host-staged base transport, P2P sums / put / push available).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6eleventh; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py -k "diagnostic_knobs" > $O/diag.txt 2>&1 || { tail -40 $O/diag.txt; exit 1; }
grep -E "PASSED|FAILED" $O/diag.txt
PE_CTOR_TRACE=1 timeout -k 10 300 python -u tools/ctor_halo_probe.py > $O/ctor.txt 2>&1 || { tail -30 $O/ctor.txt; exit 1; }
grep -E "halo path|construction|ctor (items|tuning|halo|placement)" $O/ctor.txt
PE_COMM=host PE_ALLREDUCE=p2p PE_P2P_TIMEOUT_S=60 timeout -k 10 300 python -u bench.py --gpus 4 --steps 30 --warmup 3 --grid 2048 2048 --decomp rows --no-random-solve > $O/bench4.txt 2>&1 || { tail -30 $O/bench4.txt; exit 1; }
python -c "
import json;d=json.loads([l for l in open('$O/bench4.txt') if l.startswith('{')][0]);c=d['config']
print('bench4', round(d['value'],1), d['valid'], d['converged'], d['iters_converged'], c['halo_path'], c['halo'], c['halo_candidates_us_per_sweep'])"
echo EXIT 0

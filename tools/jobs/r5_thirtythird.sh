# Round 5, thirty-third GPU call: A/B of six rows of r / p loads in flight (PE_S3_XD 6, the VGPRs the LDS scalars freed)
# against the build before it
# (.abref: HEAD 3aa2414's bench.py + extension, built here) — stamped launch
# timelines, 8192^2 / 2048^2 benches and per-rank probes, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5thirtythird; mkdir -p $O
cd $R
PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps_new.txt 2>&1 || { tail -20 $O/stamps_new.txt; exit 1; }
(cd .abref && PROBE_CFG=8:device,1:device timeout -k 10 300 python -u tools/stamp_probe.py > $O/stamps_old.txt 2>&1) || { tail -20 $O/stamps_old.txt; exit 1; }
for f in old new; do echo "== $f"; grep -h -E "^P=|state read|step scalars|walk entry|first item start|last wave exit|kernel entry \(wave\)" $O/stamps_$f.txt; done
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then D=.abref; else D=.; fi
    (cd $D && timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-random-solve > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err) || { tail -5 $O/b_${v}_$rep.err; exit 1; }
    (cd $D && timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --grid 2048 2048 --no-random-solve > $O/b2048_${v}_$rep.json 2> $O/b2048_${v}_$rep.err) || { tail -5 $O/b2048_${v}_$rep.err; exit 1; }
    python3 -c "
import json
for n in ('b_${v}_$rep','b2048_${v}_$rep'):
    d=json.loads(open('$O/%s.json'%n).read().strip().splitlines()[-1]); print(n, round(d['value'],1), 'iters', d.get('iters_converged'), 't_iterate', d.get('t_iterate_s'))"
    (cd $D && PROBE_CFG=8:device,8:4x2 timeout -k 10 120 python -u tools/block_probe.py 2>&1 | grep "us/iter" | sed "s/^/$v /")
  done
done
echo EXIT 0

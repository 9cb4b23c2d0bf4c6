# Round 6, forty-fourth GPU call: the first workgroups' share of the 8192²
# LPT layout (PE_YOUNG = rho: 1.0 default; round 5 measured 1.2+ slower) at
# 1.0 / 1.05 / 1.1, 2000-step bench, two alternating rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6fortyfourth; mkdir -p $O
cd $R
for i in 1 2; do
  for rho in 1.0 1.05 1.1; do
    PE_YOUNG=$rho timeout -k 10 200 python -u bench.py --steps 2000 --warmup 100 --no-solve > $O/b_${rho}_$i.txt 2>&1 || { tail -20 $O/b_${rho}_$i.txt; exit 1; }
    python -c "import json;d=json.loads(open('$O/b_${rho}_$i.txt').read().strip().splitlines()[-1]);p=d['config']['placement'];print('rho $rho',round(d['value'],1),p['candidates_ms_per_sweep'][p['chosen']])"
  done
done
echo EXIT 0

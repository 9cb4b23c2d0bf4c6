# Prefetch depth of the three-step march (PE_S3_XD rows of r/p, PE_S3_WD of w
# ahead; default 3/3): pe_hip builds with 6/3 and 3/6, 8192^2 and 2400x3200,
# alternating fresh processes (1500 / 3000 fixed iterations, tolerance test off).
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for b in pe_hip pe_hip_x6w3 pe_hip_x3w6; do
    for g in "8192 8192 1500" "2400 3200 3000"; do
      set -- $g
      out=$(timeout -k 10 120 bin/$b --json --quiet --max-iter $3 --no-tol $1 $2 | grep '^{') || { echo "$b failed"; exit 1; }
      echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r $b $1x$2: %.1f us/iter' % (1e6*d['t_iterate']/d['iters']))"
    done
  done
done
echo EXIT 0

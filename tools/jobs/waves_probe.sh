# Deferring-sweep grid size: default (occupancy-sized, 3 waves/SIMD) vs capped waves; per-kernel times.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/waves; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
cd /tmp && export TMPDIR=/tmp
for w in default 2048 1536 1024; do
  if [ $w = default ]; then unset PE_WAVES; else export PE_WAVES=$w; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/w$w -o run -- $BIN --json --quiet --max-iter 1000 --no-tol 8192 8192 > $O/w$w.log 2>&1 || exit 1
  echo "$w: $(grep -o '"iters_per_s": [0-9.]*' $O/w$w.log)"
done

# Is the iteration rate constant over a long run?  (fixed-iteration runs of
# increasing length, then a converging solve; per-chunk rates from --timing)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/longrun; mkdir -p $O
BIN=$GRAFT_REPO_ROOT/bin/pe_hip
( for n in 500 2000 6000; do echo "fixed $n"; timeout -k 10 100 $BIN --json --quiet --max-iter $n --no-tol 8192 8192 || exit 1; done
  echo "solve"; timeout -k 10 100 $BIN --json --quiet 8192 8192 || exit 1
  echo "fixed 6000 again"; timeout -k 10 100 $BIN --json --quiet --max-iter 6000 --no-tol 8192 8192 || exit 1
) > $O/runs.txt 2>&1 || { tail $O/runs.txt; exit 1; }
grep -E "fixed|solve|iters_per_s" $O/runs.txt | paste - - | sed -E 's/\{.*"iters": ([0-9]+).*"t_iterate": ([0-9.]+).*"iters_per_s": ([0-9.]+).*/iters=\1 t=\2 ips=\3/'
timeout -k 10 120 python - <<'PY' > $O/chunks.txt 2>&1
import time, json
import poisson_ellipse_openmp_mpi_cuda_amd as pe
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D
nat = native()
prob = pe.EllipseProblem(8192, 8192)
opt = nat.SolveOptions(); opt.check_tol = False
s = nat.DeviceSolver(prob.to_native(), D.block(8192, 8192, 1, 0), None, opt)
s.reset()
for i in range(12):
    dt = s.time_iterations(500, True)
    print(f"block {i}: {500/dt:.1f} it/s", flush=True)
PY
cat $O/chunks.txt

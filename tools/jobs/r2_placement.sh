# Placement: first allocations of fresh processes, plain vs shuffled physical
# chunks of several sizes (no search), then bench.py with the default
# (shuffled 2 MB chunks + placement search with the absolute fast-class stop).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/place
probe() {
timeout -k 10 90 python -u -c "
import sys, time; sys.path.insert(0,'.')
import poisson_ellipse_openmp_mpi_cuda_amd as pe
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D
nat=native(); prob=pe.EllipseProblem(8192,8192); opt=nat.SolveOptions(); opt.check_tol=False
keep=[]; out=[]
for i in range(2):
    s=nat.DeviceSolver(prob.to_native(), D.block(8192,8192,1,0), None, opt)
    s.reset(); s.time_iterations(20, True)
    dt=s.time_iterations(400, True)
    out.append('%.0f it/s' % (400/dt))
    keep.append(s)
print(' | '.join(out), flush=True)
"
}
for mode in "0 2" "2 2" "2 16" "2 64" "2 256"; do
  set -- $mode
  echo "PE_MALLOC=$1 chunk=$2MB (first two solvers of 3 fresh processes):"
  for r in 1 2 3; do PE_PLACEMENT_TRIES=1 PE_MALLOC=$1 PE_VMM_CHUNK_MB=$2 probe || exit 1; done
done
echo "bench.py default (3 fresh processes):"
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-solve > gpurun_out/place/bench_$r.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/place/bench_$r.json')); print(round(d['value'],1), d['config']['placement'], d['config']['construct_s'])"
done
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/place/bench_full.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/place/bench_full.json')); print('steps 20 + solve:', round(d['value'],1), d['t_solver_s'], d['t_setup_s'], d['iters_converged'], d['config']['placement'])"

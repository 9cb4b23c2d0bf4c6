# Placement experiment: plain hipMalloc vs physical chunks mapped in shuffled
# order (PE_MALLOC=2, chunk PE_VMM_CHUNK_MB) — sweep speed of several solvers
# per process (no placement search), 3 processes per mode.
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
for i in range(4):
    t0=time.perf_counter()
    s=nat.DeviceSolver(prob.to_native(), D.block(8192,8192,1,0), None, opt)
    ct=time.perf_counter()-t0
    s.reset(); s.time_iterations(20, True)
    dt=s.time_iterations(400, True)
    out.append('%.0f it/s (ctor %.2fs)' % (400/dt, ct))
    keep.append(s)
print(' | '.join(out), flush=True)
"
}
for mode in "0 2" "2 2" "2 64" "2 2" "0 2" "2 512" "1 2"; do
  set -- $mode
  echo "PE_MALLOC=$1 chunk=$2MB:"
  for r in 1 2; do PE_PLACEMENT_TRIES=1 PE_MALLOC=$1 PE_VMM_CHUNK_MB=$2 probe || exit 1; done
done

# Placement experiment: the three arrays carved from ONE allocation at relative offsets (PE_PLACEMENT=carve), 4 solvers per process, 3 processes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/place
for r in 1 2 3; do
PE_PLACEMENT=carve timeout -k 10 60 python -u -c "
import sys; sys.path.insert(0,'.')
import poisson_ellipse_openmp_mpi_cuda_amd as pe
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D
nat=native(); prob=pe.EllipseProblem(8192,8192); opt=nat.SolveOptions(); opt.check_tol=False
keep=[]
for i in range(4):
    s=nat.DeviceSolver(prob.to_native(), D.block(8192,8192,1,0), None, opt)
    print('solver',i,'carve ms/sweep', [round(x,4) for x in s.placement_ms], flush=True)
    keep.append(s)
" || exit 1
done

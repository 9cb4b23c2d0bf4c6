"""Several single-sweep solvers (one allocation each) in one process, 31
un-graphed sweeps each (1 S_0 + 30 iterations) — for per-dispatch PMC."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
prob = pe.EllipseProblem(8192, 8192)
opt = nat.SolveOptions()
opt.check_tol = False
keep = []
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    s = nat.DeviceSolver(prob.to_native(), D.block(8192, 8192, 1, 0), None, opt)
    s.reset()
    s.run_iterations(30, False)
    s.synchronize()
    keep.append(s)

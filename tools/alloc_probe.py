"""Is the single-sweep iteration rate allocation-dependent?  Creates several
solvers in one process (each its own allocation), keeps them alive, and
times a fixed number of iterations on each, twice."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

nat = native()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
prob = pe.EllipseProblem(8192, 8192)
opt = nat.SolveOptions()
opt.check_tol = False
solvers = []
for i in range(n):
    s = nat.DeviceSolver(prob.to_native(), D.block(8192, 8192, 1, 0), None, opt)
    s.reset()
    solvers.append(s)
for rep in range(1):
    for i, s in enumerate(solvers):
        dt = s.time_iterations(300, True)
        a = s.fields_address
        print(f"rep {rep} solver {i}: {300 / dt:.1f} it/s  placement_ms={[round(x, 3) for x in s.placement_ms]}",
              flush=True)

"""Placement experiment: hold a decoy allocation of G GiB, then create
solvers (kept alive) and time them."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
gib = float(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
decoy = torch.empty(int(gib * (1 << 30)), dtype=torch.uint8, device="cuda") if gib > 0 else None
prob = pe.EllipseProblem(8192, 8192)
opt = nat.SolveOptions()
opt.check_tol = False
keep = []
for i in range(n):
    s = nat.DeviceSolver(prob.to_native(), D.block(8192, 8192, 1, 0), None, opt)
    s.reset()
    s.time_iterations(20, True)
    dt = s.time_iterations(200, True)
    print(f"decoy {gib:5.1f} GiB solver {i}: {200 / dt:.1f} it/s", flush=True)
    keep.append(s)

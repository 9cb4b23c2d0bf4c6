"""Row-pitch padding vs single-sweep speed: one solver per padding (extra
doubles per plane row), physically contiguous or default allocation
(PE_MALLOC), each timed over a fixed number of iterations."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
pads = [int(x) for x in sys.argv[1].split(",")]
prob = pe.EllipseProblem(8192, 8192)
opt = nat.SolveOptions()
opt.check_tol = False
for pad in pads:
    os.environ["PE_PAD"] = str(pad)
    s = nat.DeviceSolver(prob.to_native(), D.block(8192, 8192, 1, 0), None, opt)
    s.reset()
    s.time_iterations(20, True)
    dt = s.time_iterations(200, True)
    print(f"pad {pad:5d}: {200 / dt:.1f} it/s", flush=True)
    del s

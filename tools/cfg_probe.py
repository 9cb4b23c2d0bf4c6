"""Time the 8192² single sweep under several PE_* configurations in ONE
process (each solver its own allocation; set PE_MALLOC=1 outside for the
deterministic, physically contiguous placement).
    python tools/cfg_probe.py "PE_TI=8,PE_ORDER=0" "PE_TI=16,PE_ORDER=2" ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
grid = int(os.environ.get("PROBE_GRID", "8192"))
prob = pe.EllipseProblem(grid, grid)
opt = nat.SolveOptions()
opt.check_tol = False
base = dict(os.environ)
for spec in sys.argv[1:]:
    env = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
    for key in [k for k in os.environ if k.startswith("PE_") and k not in base]:
        del os.environ[key]
    os.environ.update(env)
    s = nat.DeviceSolver(prob.to_native(), D.block(grid, grid, 1, 0), None, opt)
    s.reset()
    s.time_iterations(20, True)
    dt = s.time_iterations(200, True)
    print(f"{spec:40s} {200 / dt:8.1f} it/s  ti={s.ti} blocks={s.blocks}", flush=True)
    del s

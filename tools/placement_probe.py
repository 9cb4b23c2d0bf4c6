"""Memory-placement spread of one rank's block: fresh solvers, the placement
search forced with PE_PLACEMENT_TRIES (else the solver's own rule: a search
from 24 M nodes per block), each printing its candidates' ms
per sweep and the chosen one, then 300 timed iterations of the solver as
constructed.  One rank's block of a P-rank split of 8192² on one GPU (delay
transport, zero delays: no communication cost).

    PROBE_CFG=8:rows,4:rows PROBE_REPS=3 python tools/placement_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
nat.set_device(0)
os.environ.setdefault("PE_HALO", "exchange")
os.environ.setdefault("PE_OVERLAP", "0")
M = N = 8192
for spec in os.environ.get("PROBE_CFG", "8:rows,4:rows").split(","):
    P, sp = int(spec.split(":")[0]), spec.split(":")[1]
    blk = nat.decompose(M, N, D.grid(P, M, N, sp), P // 2)
    for rep in range(int(os.environ.get("PROBE_REPS", "3"))):
        comm = nat.make_delay_comm(P, 0.0, 0.0, True)
        opt = nat.SolveOptions()
        opt.check_tol = False
        s = nat.DeviceSolver(pe.EllipseProblem(M, N).to_native(), blk, comm, opt)
        s.reset()
        s.time_iterations(30, False)
        us = s.time_iterations(300, False) / 300 * 1e6
        print(f"P={P} {sp} block {blk.nx}x{blk.ny} rep {rep}: placement ms/sweep {[round(x, 4) for x in s.placement_ms]} "
              f"chosen {s.placement_choice} (search {s.placement_s:.3f} s) -> {us:.1f} us/iter, ti {s.ti}", flush=True)
        del s, comm

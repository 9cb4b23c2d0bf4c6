"""Construction cost of the halo-path choice (≤ 10 ms at
the 8-rank slab of 8192²).  One rank's block, delay transport (0 / 0 µs),
the loopback put and push so that all five candidates are timed; run with
PE_CTOR_TRACE=1 — the "halo path" phase of the construction trace is the
choice (every candidate's 2 + 4 sweeps, the two finalists again, re-layouts)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
nat.set_device(0)
os.environ.setdefault("PE_PUT_LOOPBACK", "1")
os.environ.setdefault("PE_PUSH_LOOPBACK", "1")
for spec in os.environ.get("PROBE_CFG", "8:rows,8:4x2,2:rows").split(","):
    P, sp = int(spec.split(":")[0]), spec.split(":")[1]
    M = N = int(os.environ.get("PROBE_N", "8192"))
    blk = nat.decompose(M, N, D.grid(P, M, N, sp), P // 2)
    for rep in range(2):
        comm = nat.make_delay_comm(P, 0.0, 0.0, True)
        t0 = time.perf_counter()
        s = nat.DeviceSolver(pe.EllipseProblem(M, N).to_native(), blk, comm, nat.SolveOptions())
        dt = time.perf_counter() - t0
        print(f"{P} {sp} block {blk.nx}x{blk.ny} construction {dt * 1e3:.1f} ms; chosen {s.halo_path}; "
              f"{len(s.halo_candidates)} timings", flush=True)
        del s, comm

"""Rows-per-item sweep on ONE solver (one memory placement, so candidates
compare without the placement lottery): construct once with room for the
smallest item height, then relayout(ti) and time a fixed number of
iterations for each candidate.

    PROBE_GRIDS=8192x8192,2048x2048 PROBE_TI=24,32,40,48 PROBE_ALGO=3 python tools/ti_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
grids = [tuple(int(v) for v in g.split("x")) for g in os.environ.get("PROBE_GRIDS", "8192x8192").split(",")]
tis = [int(t) for t in os.environ.get("PROBE_TI", "24,32,40,48").split(",")]
algo = int(os.environ.get("PROBE_ALGO", "3"))
iters = int(os.environ.get("PROBE_ITERS", "400"))
reps = int(os.environ.get("PROBE_REPS", "2"))
os.environ["PE_TI"] = str(min(tis))  # item-sum slots for the smallest height
for M, N in grids:
    prob = pe.EllipseProblem(M, N)
    opt = nat.SolveOptions()
    opt.check_tol = False
    opt.algo = algo
    s = nat.DeviceSolver(prob.to_native(), D.block(M, N, 1, 0), None, opt)
    res = {t: [] for t in tis}
    for _ in range(reps):
        for t in tis:
            s.relayout(t)
            s.reset()
            s.time_iterations(40, False)
            res[t].append(s.time_iterations(iters, False) / iters * 1e6)
    best = min(tis, key=lambda t: min(res[t]))
    print(f"{M}x{N} algo {algo} placement {[round(x, 4) for x in s.placement_ms]}: " +
          "  ".join(f"ti {t}: {min(res[t]):.1f}" for t in tis) + f"  us/iter  -> best {best}", flush=True)
    del s

"""Short timed windows on one solver (the driver's bench shape: reset, then
K iterations from a fresh solve), graph-replayed vs eager, repeated, to see
what a 20-iteration window costs beyond 20 × the steady per-iteration time.

    PROBE_GRID=8192x8192 PROBE_K=20,18,21 PROBE_REPS=4 python tools/window_probe.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
M, N = (int(v) for v in os.environ.get("PROBE_GRID", "8192x8192").split("x"))
ks = [int(k) for k in os.environ.get("PROBE_K", "20,18,21").split(",")]
reps = int(os.environ.get("PROBE_REPS", "4"))
idle_ms = float(os.environ.get("PROBE_IDLE_MS", "0"))
prob = pe.EllipseProblem(M, N)
opt = nat.SolveOptions()
opt.check_tol = False
s = nat.DeviceSolver(prob.to_native(), D.block(M, N, 1, 0), None, opt)
print(f"{M}x{N}: steps/sweep {s.sweep_steps}, placement {[round(x, 4) for x in s.placement_ms]} "
      f"chosen {s.placement_choice}", flush=True)
for k in ks:
    s.prepare_graphs(k)
for rep in range(reps):
    for k in ks:
        for graph in (True, False):
            s.reset()
            s.synchronize()
            if idle_ms > 0:
                time.sleep(idle_ms * 1e-3)
            t0 = time.perf_counter()
            s.run_iterations(k, graph)
            s.synchronize()
            dt = time.perf_counter() - t0
            print(f"  rep {rep} K {k:3d} {'graph' if graph else 'eager'}: {dt * 1e3:7.3f} ms  "
                  f"{dt / k * 1e6:7.1f} us/iter  {k / dt:7.1f} it/s", flush=True)

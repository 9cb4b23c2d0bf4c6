"""Does a short timed window right after construction run slower than the
same window later?  One 8192² solver (bench.py's construction, placement
search included), then the driver-shaped window (reset, 20 timed steps)
repeated after increasing idle times, and a 20-step window right after a
long warm-up — µs per step each.

    python tools/settle_probe.py            (PROBE_STEPS=20 PROBE_WAITS=0,0.2,1,3)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
steps = int(os.environ.get("PROBE_STEPS", "20"))
waits = [float(x) for x in os.environ.get("PROBE_WAITS", "0,0.2,1,3").split(",")]
prob = pe.EllipseProblem(8192, 8192)
blk = D.block(8192, 8192, 1, 0, "device")
opt = nat.SolveOptions()
opt.check_tol = False
t_c = time.perf_counter()
s = nat.DeviceSolver(prob.to_native(), blk, None, opt)
print(f"construct {time.perf_counter() - t_c:.3f} s, placement {[round(x, 4) for x in s.placement_ms]}", flush=True)


def window(tag):
    s.reset()
    s.synchronize()
    t0 = time.perf_counter()
    s.run_iterations(steps, False)
    s.synchronize()
    dt = time.perf_counter() - t0
    print(f"  {tag}: {dt / steps * 1e6:7.1f} us/step ({steps / dt:7.1f} it/s)", flush=True)


s.reset()
s.run_iterations(5, False)
s.synchronize()
window("right after construction")
for w in waits:
    time.sleep(w)
    window(f"after {w:.1f} s idle")
s.reset()
s.run_iterations(600, False)
s.synchronize()
window("after 600 warm-up iterations")

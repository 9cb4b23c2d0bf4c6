"""Does the construction's short timing of a halo path predict its steady
state?  One rank's block of an 8-rank split of 8192² on one GPU (delay
transport, zero delays, loopback copies): the solver constructed with the
exchange arms as candidates (PE_HALO=exchange), then each arm switched to
(set_halo_path) and timed both ways — time_halo_path(4) (the construction's
measure: 2 + 4 sweeps after a reset) and time_iterations over 300 iterations.
A freshly constructed solver with the overlap forced is timed as well."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
GM, GN = (int(v) for v in os.environ.get("PROBE_GRID", "8192x8192").split("x"))
P = int(os.environ.get("PROBE_P", "8"))
prob = pe.EllipseProblem(GM, GN)
os.environ["PE_HALO"] = "exchange"
for spec in os.environ.get("PROBE_SPEC", "rows,4x2").split(","):
    blk = nat.decompose(GM, GN, D.grid(P, GM, GN, spec), P // 2)
    os.environ.pop("PE_OVERLAP", None)
    opt = nat.SolveOptions()
    opt.check_tol = False
    comm = nat.make_delay_comm(P, 0.0, 0.0, True)
    s = nat.DeviceSolver(prob.to_native(), blk, comm, opt)
    print(f"{spec} P={P}: chosen {s.halo_path}; candidates {[(n, round(t, 1)) for n, t in s.halo_candidates]}", flush=True)
    for ov in (False, True, False, True):
        s.set_halo_path("exchange", ov)
        short = s.time_halo_path(4) * 1e3 / 3
        s.reset()
        s.time_iterations(6, False)
        long_ = s.time_iterations(300, False) / 300 * 1e6
        print(f"    overlap={ov} ({s.overlap}, boundary items {s.layout_boundary}): short {short:6.1f} us/iter, "
              f"300 iterations {long_:6.1f} us/iter", flush=True)
    del s, comm
    os.environ["PE_OVERLAP"] = "1"
    for rep in range(3):  # fresh solvers, one after the other (each takes the pooled stream pair)
        comm = nat.make_delay_comm(P, 0.0, 0.0, True)
        s = nat.DeviceSolver(prob.to_native(), blk, comm, opt)
        short = s.time_halo_path(4) * 1e3 / 3
        s.reset()
        s.time_iterations(6, False)
        long_ = s.time_iterations(300, False) / 300 * 1e6
        print(f"    forced at construction ({rep}): {s.halo_path} (boundary items {s.layout_boundary}): short {short:6.1f}, "
              f"300 iterations {long_:6.1f} us/iter", flush=True)
        del s, comm

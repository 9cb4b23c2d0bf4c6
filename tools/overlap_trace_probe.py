"""Kernel-trace companion of overlap_steady_probe.py: fresh solvers with the
overlap forced (one rank's block of the 8-rank slab of 8192², delay
transport, zero delays, loopback copies), 60 iterations each, separated by
20 ms idle gaps so `tools/rocpd_summary.py --segments 5` gives one table per
solver (sweep / kWaitSig / copy / unpack durations).  Run under
`rocprofv3 --kernel-trace`."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
nat.set_device(0)
M = N = 8192
P, spec = 8, os.environ.get("PROBE_SPEC", "rows")
blk = nat.decompose(M, N, D.grid(P, M, N, spec), P // 2)
os.environ["PE_HALO"] = os.environ.get("PROBE_HALO", "exchange")
if os.environ["PE_HALO"] == "put":  # (the delay transport maps no peer inboxes: the loopback put)
    os.environ["PE_PUT_LOOPBACK"] = "1"
os.environ["PE_OVERLAP"] = "1"
for rep in range(int(os.environ.get("PROBE_REPS", "4"))):
    comm = nat.make_delay_comm(P, 0.0, 0.0, True)
    opt = nat.SolveOptions()
    opt.check_tol = False
    s = nat.DeviceSolver(pe.EllipseProblem(M, N).to_native(), blk, comm, opt)
    s.synchronize()
    time.sleep(0.02)
    s.reset()
    dt = s.time_iterations(60, False)
    print(f"rep {rep}: {s.halo_path}: {dt / 60 * 1e6:.1f} us/iter  (rows per item {s.ti}, layout {s.layout_name}, "
          f"tuning {[(r, round(m, 4)) for r, m in zip(s.ti_tuning_rows, s.ti_tuning_ms)]}; "
          f"halo candidates {[(n, round(t, 1)) for n, t in s.halo_candidates]})", flush=True)
    s.synchronize()
    time.sleep(0.02)
    del s, comm

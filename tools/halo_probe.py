"""The construction's halo-path choice on one GPU.

One GPU runs the block of one rank of a P-rank decomposition with the
loopback forms of every halo path: the delay transport stands in for the
comm's exchange (a stream-ordered busy wait of `exchange_us` per halo phase,
`allreduce_us` per cross-rank sum, then a device copy of every message into
its own receive buffer), PE_PUT_LOOPBACK=1 runs the peer-put kernel into the
rank's own inbox, PE_PUSH_LOOPBACK=1 the sweep's push into its own receive
buffer.  For each delay pair the solver's own choice (DeviceSolver::
choose_halo_path) is printed with every candidate's µs per sweep, then the
chosen path is timed over 300 iterations, and (PROBE_EACH=1) every forced path
too.  What one GPU cannot show is the xGMI leg of the put / push (loopback
stores stay on the device) and the real RCCL latency — the delays model them.

    python tools/halo_probe.py [exchange_us allreduce_us ...]
    PROBE_CFG=8:rows,4:rows,8:4x2 PROBE_GRID=8192x8192 PROBE_EACH=1
    PROBE_HALO=exchange  (the auto run chooses among the exchange arms only:
                          the projections' model — the loopback put / push pay
                          no xGMI time, the delayed exchange does)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
args = [float(x) for x in sys.argv[1:]] or [0.0, 0.0, 15.0, 8.0]
delays = list(zip(args[0::2], args[1::2]))
configs = [(int(c.split(":")[0]), c.split(":")[1]) for c in os.environ.get("PROBE_CFG", "8:rows,4:rows,8:4x2").split(",")]
GM, GN = (int(v) for v in os.environ.get("PROBE_GRID", "8192x8192").split("x"))
each = os.environ.get("PROBE_EACH", "0") == "1"
iters = int(os.environ.get("PROBE_ITERS", "300"))
prob = pe.EllipseProblem(GM, GN)
os.environ["PE_PUT_LOOPBACK"] = "1"
os.environ["PE_PUSH_LOOPBACK"] = "1"


def run(P, blk, ex, ar, halo=None, ov=None):
    for k, v in (("PE_HALO", halo), ("PE_OVERLAP", ov)):
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    opt = nat.SolveOptions()
    opt.check_tol = False
    comm = nat.make_delay_comm(P, ex, ar, True)
    t0 = time.perf_counter()
    s = nat.DeviceSolver(prob.to_native(), blk, comm, opt)
    ctor = time.perf_counter() - t0
    s.reset()
    s.time_iterations(30, False)
    dt = s.time_iterations(iters, False)
    out = (s.halo_path, list(s.halo_candidates), dt / iters * 1e6, ctor)
    del s, comm
    return out


for P, spec in configs:
    g = D.grid(P, GM, GN, spec)
    rank = P // 2
    blk = nat.decompose(GM, GN, g, rank)
    for ex, ar in delays:
        path, cands, us, ctor = run(P, blk, ex, ar, os.environ.get("PROBE_HALO"))
        cs = ", ".join(f"{n} {t:.1f}" for n, t in cands)
        print(f"P={P} {g.Px}x{g.Py} rank {rank} block {blk.nx}x{blk.ny} delays ex={ex:5.1f} ar={ar:5.1f} us: "
              f"chosen {path}: {us:7.1f} us/iter (construction {ctor * 1e3:.0f} ms) | candidates us/sweep: {cs}",
              flush=True)
        if each:
            for halo, ov in (("exchange", "0"), ("exchange", "1"), ("put", "0"), ("put", "1"), ("push", "0")):
                if halo == "push" and g.Py != 1:
                    continue
                p2, _, us2, _ = run(P, blk, ex, ar, halo, ov)
                print(f"    forced {p2:32s} {us2:7.1f} us/iter", flush=True)

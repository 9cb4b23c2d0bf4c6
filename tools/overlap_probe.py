"""How much communication latency does the halo/interior overlap hide?
One GPU runs the block of one rank of a multi-GPU decomposition with a
timing-only transport (stream-ordered busy waits of fixed length stand in
for the RCCL exchange and allreduce), with PE_OVERLAP=0 and 1
(PROBE_OV=0,1,1::2 → overlap[::PE_OV_DEBUG]; 8 blocks stay free for the
halo stream).

    python tools/overlap_probe.py [exchange_us allreduce_us]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
ex_us = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
ar_us = float(sys.argv[2]) if len(sys.argv) > 2 else 12.0
graph = os.environ.get("PROBE_GRAPH", "1") == "1"
configs = [(int(c.split(":")[0]), c.split(":")[1]) for c in os.environ.get("PROBE_CFG", "2:aspect,4:aspect,8:aspect,8:rows").split(",")]
GM, GN = (int(v) for v in os.environ.get("PROBE_GRID", "8192x8192").split("x"))
prob = pe.EllipseProblem(GM, GN)
for P, spec in configs:
    g = D.grid(P, GM, GN, spec)
    rank = P // 2
    blk = nat.decompose(GM, GN, g, rank)
    for delays in [(0.0, 0.0), (ex_us, ar_us)]:
        for ov in os.environ.get("PROBE_OV", "0,1:8").split(","):
            os.environ["PE_OVERLAP"] = ov.split(":")[0]
            os.environ["PE_OV_DEBUG"] = ov.split(":")[2] if ov.count(":") > 1 else "0"
            opt = nat.SolveOptions()
            opt.check_tol = False
            comm = nat.make_delay_comm(P, delays[0], delays[1])
            s = nat.DeviceSolver(prob.to_native(), blk, comm, opt)
            s.reset()
            s.time_iterations(20, graph)
            dt = s.time_iterations(300, graph)
            print(f"P={P} {g.Px}x{g.Py} rank {rank} block {blk.nx}x{blk.ny}  delays ex={delays[0]:4.0f} ar={delays[1]:4.0f} "
                  f"us  overlap={ov} ({s.overlap}):  {dt / 300 * 1e6:7.1f} us/iter", flush=True)
            del s, comm

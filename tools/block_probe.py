"""Per-rank block efficiency: one GPU runs the block of one rank of a P-rank
decomposition of 8192² (timing-only transport with zero delays, overlap off,
eager) under a list of kernel configurations.

    PROBE_CFG=8:aspect,4:aspect PROBE_ENV="PE_TI=8 PE_ORDER=0;PE_TI=16 PE_ORDER=3" python tools/block_probe.py
    PROBE_RANKS=all (every rank's block in turn; default: rank P//2)
    PE_PUSH_LOOPBACK=1: row slabs run the halo-push kernel, pushing into their own receive buffer
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
configs = [(int(c.split(":")[0]), c.split(":")[1]) for c in os.environ.get("PROBE_CFG", "8:aspect").split(",")]
envs = [e.strip() for e in os.environ.get("PROBE_ENV", "").split(";")]
iters = int(os.environ.get("PROBE_ITERS", "400"))
GM, GN = (int(v) for v in os.environ.get("PROBE_GRID", "8192x8192").split("x"))
prob = pe.EllipseProblem(GM, GN)
os.environ["PE_OVERLAP"] = "0"
# PROBE_RANKS: "mid" (default, rank P//2), "all", or a comma list
rsel = os.environ.get("PROBE_RANKS", "mid")
for P, spec in configs:
    g = D.grid(P, GM, GN, spec)
    ranks = [P // 2] if rsel == "mid" else list(range(P)) if rsel == "all" else [int(r) for r in rsel.split(",")]
    for rank in ranks:
        blk = nat.decompose(GM, GN, g, rank)
        for env in envs:
            kv = dict(x.split("=") for x in env.split()) if env else {}
            saved = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            opt = nat.SolveOptions()
            opt.check_tol = False
            comm = nat.make_delay_comm(P, 0.0, 0.0) if P > 1 else None
            s = nat.DeviceSolver(prob.to_native(), blk, comm, opt)
            s.reset()
            s.time_iterations(20, False)
            dt = s.time_iterations(iters, False)
            tune = " ".join(f"{x * 1e3:.1f}" for x in s.ti_tuning_ms)
            print(f"P={P} {g.Px}x{g.Py} rank {rank} block {blk.nx}x{blk.ny} [{env or 'default'}]: {dt / iters * 1e6:7.1f} us/iter "
                  f"({blk.nx * blk.ny / (dt / iters) / 1e9:6.2f} Gpt/s)  ti {s.ti}" + (f"  tuning us/sweep [{tune}]" if tune else "")
                  + (f"  push {s.push_status}" if os.environ.get("PE_PUSH_LOOPBACK") == "1" else ""),
                  flush=True)
            del s, comm
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

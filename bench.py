#!/usr/bin/env python3
"""Headline benchmark: PCG iterations/s on the 8192×8192 fictitious-domain
Poisson problem (BASELINE.json: "PCG iters/sec + T_solver, 8192x8192 grid at
1/2/4/8 MI355X; L2 err vs analytic"), fp64, δ = 1e-6.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 8192]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

A *step* is one full PCG iteration of the global solve on N GPUs (the
single-sweep kernel with its 7 sums summed over ranks inside the sweep over
xGMI P2P, and the halo rows — row-slab blocks — pushed by the same sweep into
the neighbours' receive buffers, or exchanged through RCCL otherwise).  The timed region runs exactly K steps from the start of a fresh
solve (w⁰ = 0, as the reference) with the convergence test switched off so
every step does full work; it is bracketed by a barrier + device synchronise
on both sides and the max over ranks is reported (each rank's clock stops at
its closing device synchronise, before the closing CPU barrier: the ranks are
coupled every iteration by the in-sweep sums, so the max over ranks is the
job's time, without the gloo barrier's ~0.1-0.3 ms, which at 8 ranks would be
≈10 % of a 20-step window).  `value` = job-wide PCG
iterations/s (the grid is fixed → strong scaling).  Outside the timed region
the script also runs one complete solve to convergence and reports T_solver,
its iteration count and the L2 error against the analytic solution.

vs_baseline: the reference never ran 8192²; BASELINE.md §1b extrapolates one
P100 to ≈270 s for its 5889 iterations = 21.8 iterations/s, which is the
number used here (stated in the JSON as `baseline`).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import dist as PD  # noqa: E402

P100_ITERS_PER_S_8192 = 5889 / 270.0  # BASELINE.md §1b extrapolation (1× P100)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--grid", type=int, nargs="+", default=[8192, 8192])
    ap.add_argument("--decomp", default="device", help="device | aspect | reference | rows | cols | <Px>x<Py>")
    ap.add_argument("--no-solve", action="store_true", help="skip the (untimed) full solve")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--algo", default="auto", choices=("auto", "classic", "fused"))
    ap.add_argument("--launch", default="graph", choices=("graph", "eager"),
                    help="timed steps replayed from instantiated hipGraphs (default) or launched eagerly")
    a = ap.parse_args()
    M, N = (a.grid[0], a.grid[-1])

    rank, world, local = PD.env_rank_world()
    if world != a.gpus:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    nat = native()
    if nat.device_count() < 1:
        print("[bench] no HIP device visible", file=sys.stderr)
        return 2
    ctx = None
    comm = None
    cpu_group = None
    if world > 1:
        ctx = PD.init()
        import torch.distributed as dist

        cpu_group = dist.new_group(backend="gloo")
        comm = PD.rccl_comm(ctx)
    else:
        nat.set_device(0)
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))

    prob = EllipseProblem(M, N)
    P = prob.to_native()
    blk = D.block(M, N, world, rank, a.decomp)
    opt = nat.SolveOptions()
    opt.check_tol = False  # fixed work per step in the timed region
    opt.variant = a.variant
    opt.algo = {"auto": 0, "classic": 1, "fused": 2}[a.algo]
    solver = nat.DeviceSolver(P, blk, comm, opt)

    def barrier():
        if world > 1:
            import torch.distributed as dist

            dist.barrier(group=cpu_group)

    def maxval(x: float) -> float:
        if world == 1:
            return x
        import torch.distributed as dist

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=cpu_group)
        return float(t[0])

    # warmup: first-touch / RCCL connections, then instantiate every chunk
    # graph the timed run will launch (no capture inside the timed region)
    use_graph = a.launch == "graph"
    solver.reset()
    if a.warmup > 0:
        solver.run_iterations(a.warmup, use_graph)
    solver.synchronize()
    if use_graph:
        solver.prepare_graphs(a.steps)
    solver.reset()  # the timed steps start a fresh solve (w⁰ = 0)
    solver.synchronize()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    solver.run_iterations(a.steps, use_graph)
    solver.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()  # this rank's steps are done; the slowest rank is the job's time (max below)
    barrier()
    dt = maxval(t1 - t0)
    st = solver.state()
    valid = int(st["status"]) == 0 and int(st["iter"]) == a.steps

    extra = {}
    if not a.no_solve:
        # the full solve runs on the same solver (one construction, one
        # placement search; its T_solver still spans that construction)
        solver.set_check_tol(True)
        barrier()
        res = solver.solve()
        tm = res.timers
        extra = dict(t_solver_s=maxval(tm["solver"]), t_setup_s=maxval(tm["setup"]), t_iterate_s=maxval(tm["iterate"]),
                     t_breakdown_s={k: maxval(tm[k]) for k in ("gpu", "dot", "halo", "reduce", "copy")},
                     iters_converged=int(res.iters), converged=bool(res.converged),
                     l2_err=float(res.l2_err), max_err=float(res.max_err),
                     solve_iters_per_s=float(res.iters) / maxval(tm["iterate"]))

    ips = a.steps / dt
    out = {
        "metric": "pcg_iters_per_sec_8192x8192" if (M, N) == (8192, 8192) else f"pcg_iters_per_sec_{M}x{N}",
        "value": ips,
        "unit": "PCG iterations/s (global solve)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1000.0 * dt / a.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": ips / P100_ITERS_PER_S_8192 if (M, N) == (8192, 8192) else None,
        "baseline": "1x P100 extrapolated 21.8 it/s (BASELINE.md 1b: 5889 iters in ~270 s)",
        "dtype": "fp64",
        "data": "synthetic: analytic test problem (F=1 on x^2+4y^2<1), w0=0, tol 1e-6 (tol check off in timed steps)",
        "config": {
            "model": "poisson-ellipse fictitious-domain Jacobi-PCG",
            "grid": [M, N],
            "unknowns": (M - 1) * (N - 1),
            "global_batch": 1,
            "seq_len": None,
            "parallelism": (f"2d-decomp {blk.Px}x{blk.Py} "
                            + ("(xGMI halo push + P2P sums)" if solver.halo_push else "(RCCL halo)"))
            if world > 1 else "single-gpu",
            "points_per_s": ips * (M - 1) * (N - 1),
            "algo": "single-sweep (1 kernel, 1 allreduce / iter)" if solver.fused else "classic (2 kernels, 2 allreduces / iter)",
            "decomposition": {"spec": a.decomp, "Px": blk.Px, "Py": blk.Py, "block": [blk.nx, blk.ny]},
            "transport": comm.name if comm is not None else "none",
            "allreduce": ("in-sweep P2P over xGMI" if solver.xr else "launch per iteration") if world > 1 else "none",
            "halo": ("in-sweep xGMI push (graph-captured)" if solver.halo_push else
                     ("exchange: " + comm.name)) if world > 1 else "none",
            "overlap": bool(solver.overlap),
            "exchange_us_measured": round(solver.exchange_us, 2),
            "item_order": "dynamic per-XCD queue" if solver.order == 3 else "static LPT layout",
            "rows_per_item": solver.ti,
            "rows_per_item_tuning_ms": [round(x, 4) for x in solver.ti_tuning_ms],
            "resident": bool(solver.resident),
            "chunk": solver.chunk,
            "launch": a.launch,
            "placement": {"candidates_ms_per_sweep": [round(x, 4) for x in solver.placement_ms],
                          "chosen": solver.placement_choice, "search_s": round(solver.placement_s, 3)},
            "construct_s": round(solver.construct_s, 3),
        },
        "valid": valid,
    }
    out.update(extra)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if ctx is not None:
        barrier()
    if not valid or (extra and not extra.get("converged", False)):
        print(f"[bench] invalid run: status {int(st['status'])}, {int(st['iter'])} of {a.steps} steps", file=sys.stderr)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Headline benchmark: PCG iterations/s on the 8192×8192 fictitious-domain
Poisson problem (BASELINE.json: "PCG iters/sec + T_solver, 8192x8192 grid at
1/2/4/8 MI355X; L2 err vs analytic"), fp64, δ = 1e-6.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 8192]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Launch: under torchrun (WORLD_SIZE set) this process is one rank and
`--gpus` must equal WORLD_SIZE.  Without a launcher, `--gpus N > 1` starts
the N ranks itself: it checks (without initialising HIP) that N GPUs are
visible — fewer is an error, never a silent 1-rank run — and runs
`torch.distributed.run --nproc-per-node N bench.py …` as a child process,
relaying rank 0's JSON line and returning the job's exit status (the
reference's stage 4 runs as N MPI ranks on N GPUs,
stage4-mpi+cuda/poisson_mpi_cuda2.cu:986-990).

A *step* is one full PCG iteration of the global solve on N GPUs (the
three-step sweep advances three per launch, its 19 sums summed over ranks
inside the sweep over xGMI P2P; the halo path — the comm's RCCL exchange,
the peer-put kernel or the sweep's own push, with or without the
halo/interior overlap — is the one the solver's construction timed fastest
on this job's transport, reported as `halo_path` with every candidate's
time; K steps with 3 ∤ K end with a partial sweep).  The
timed region runs exactly K steps from the start of a fresh solve (w⁰ = 0, as
the reference) with the convergence test switched off so every step does full
work; it is bracketed by a barrier + device synchronise on both sides and the
max over ranks is reported (each rank's clock stops at its closing device
synchronise, before the closing CPU barrier: the ranks are coupled every
iteration by the in-sweep sums, so the max over ranks is the job's time,
without the gloo barrier's ~0.1-0.3 ms, which at 8 ranks would be ≈10 % of a
20-step window).  `value` = job-wide PCG iterations/s (the grid is fixed →
strong scaling).  Outside the timed region the script also runs one complete
solve to convergence (w⁰ = 0: T_solver, iterations, L2 error against the
analytic solution, timer breakdown incl. the cross-rank wait) and one with
the BASELINE's random-init w⁰ (`random_init`; the reference has no random
init, so its iteration count is parity-unpinned).

Every multi-rank wait is bounded: PE_P2P_TIMEOUT_S (default 30 s here) on
the in-sweep cross-rank sums, PE_WATCHDOG_S (default 60 s here) on every host
wait of the timed region and the solves (the communicator is aborted and the
rank exits non-zero; torchrun then ends the job).

vs_baseline: the reference never ran 8192²; BASELINE.md §1b extrapolates one
P100 to ≈270 s for its 5889 iterations = 21.8 iterations/s, which is the
number used here (stated in the JSON as `baseline`).
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

P100_ITERS_PER_S_8192 = 5889 / 270.0  # BASELINE.md §1b extrapolation (1× P100)


def parse_args(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--warmup-s", type=float, default=0.25,
                    help="the warm-up lasts at least this long (GPU clocks ramp up under load; 0: exactly --warmup steps)")
    ap.add_argument("--grid", type=int, nargs="+", default=[8192, 8192])
    ap.add_argument("--decomp", default="device", help="device | aspect | reference | rows | cols | <Px>x<Py>")
    ap.add_argument("--no-solve", action="store_true", help="skip the (untimed) full solves")
    ap.add_argument("--no-random-solve", action="store_true", help="skip the (untimed) random-init solve")
    ap.add_argument("--seed", type=int, default=1234, help="random-init w0 seed")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--algo", default="auto", choices=("auto", "classic", "fused", "two-step", "three-step"),
                    help="sweep kernel (auto: three-step beyond the LDS-resident kernel's blocks); two-step runs "
                         "whole two-iteration sweeps only, so it needs an even --steps")
    # eager by default: a 20-step window launched eagerly took 5.29-5.41 ms
    # against 5.30-5.85 ms replayed from its chunk graph (the first replay of
    # a window sometimes paid ~0.5 ms more: profiles/r3_window.txt)
    ap.add_argument("--launch", default="eager", choices=("graph", "eager"),
                    help="timed steps launched eagerly (default) or replayed from instantiated hipGraphs")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _visible_gpus() -> int:
    """GPUs this process could open, without initialising HIP in it (the ranks
    are separate processes; torch.cuda.device_count() does not initialise the
    device on this image)."""
    import torch

    return int(torch.cuda.device_count())


def launch_ranks(a, argv) -> int:
    """Parent of an N-rank run started without a launcher."""
    n = _visible_gpus()
    shared = os.environ.get("PE_COMM") == "host"  # test transport: ranks may share one GPU
    if n < 1 or (n < a.gpus and not shared):
        print(f"[bench] --gpus {a.gpus} needs {a.gpus} visible GPUs, this node has {n}", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

    def _die_with_parent():  # the launcher never outlives this process
        try:
            import ctypes

            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except OSError:
            pass

    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, start_new_session=True,
                         preexec_fn=_die_with_parent)

    def _forward(sig, _frame):
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            pass

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, _forward)
    assert p.stdout is not None
    for line in p.stdout:  # rank 0's JSON line → stdout; anything else → stderr
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    rc = p.wait()
    if rc != 0:
        print(f"[bench] {a.gpus}-rank job failed (exit {rc})", file=sys.stderr)
    return rc


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a, argv)

    # bounded multi-rank waits (read by the comm / solver constructors)
    os.environ.setdefault("PE_P2P_TIMEOUT_S", "30")
    os.environ.setdefault("PE_WATCHDOG_S", "60")

    import torch

    from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, native
    from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D
    from poisson_ellipse_openmp_mpi_cuda_amd.parallel import dist as PD

    M, N = (a.grid[0], a.grid[-1])
    rank, world, local = PD.env_rank_world()
    if world != a.gpus:
        print(f"[bench] --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    nat = native()
    ndev = nat.device_count()
    if ndev < 1:
        print("[bench] no HIP device visible", file=sys.stderr)
        return 2
    if world > ndev and os.environ.get("PE_COMM") != "host":
        print(f"[bench] {world} ranks but only {ndev} GPUs visible (one GPU per rank)", file=sys.stderr)
        return 2
    ctx = None
    comm = None
    cpu_group = None
    if world > 1:
        ctx = PD.init()
        import torch.distributed as dist

        cpu_group = dist.new_group(backend="gloo")
        comm = PD.rccl_comm(ctx)
        if comm.size != world:
            print(f"[bench] communicator has {comm.size} ranks, WORLD_SIZE={world}", file=sys.stderr)
            return 2
    else:
        nat.set_device(0)
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))

    prob = EllipseProblem(M, N)
    P = prob.to_native()
    blk = D.block(M, N, world, rank, a.decomp)
    opt = nat.SolveOptions()
    opt.check_tol = False  # fixed work per step in the timed region
    opt.variant = a.variant
    opt.algo = {"auto": 0, "classic": 1, "fused": 2, "two-step": 3, "three-step": 4}[a.algo]
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

    def gather(obj):
        if world == 1:
            return [obj]
        import torch.distributed as dist

        out = [None] * world
        dist.all_gather_object(out, obj, group=cpu_group)
        return out

    dev = nat.current_device()
    me = {"rank": rank, "local_rank": local, "device": dev, "pci_bus_id": nat.device_pci_bus_id(dev),
          "block": [blk.nx, blk.ny],
          "placement_ms_per_sweep": [round(x, 4) for x in solver.placement_ms],
          "placement_chosen": solver.placement_choice, "construct_s": round(solver.construct_s, 3),
          # first cross-device run diagnostics: peer access toward every rank
          # (1/0, -1 same device), the neighbours, what each self-tested
          # transport set-up decided and what the sweep finally uses
          "neighbors": {d: int(blk.nbr[i]) for i, d in enumerate(("left", "right", "down", "up")) if blk.nbr[i] >= 0},
          "peer_access": {str(r): int(v) for r, v in enumerate(solver.peer_access)},
          "p2p_sum_setup": nat.p2p_setup_status(), "halo_push": solver.push_status, "halo_put": solver.put_status,
          "sums": solver.xr_status}
    ranks_info = gather(me)

    # warmup: first-touch / RCCL connections, then (--launch graph)
    # instantiate every chunk graph the timed run will launch (no capture
    # inside the timed region)
    use_graph = a.launch == "graph"
    sweep = int(solver.sweep_steps) if int(solver.sweep_steps) == 2 else 1

    def whole_sweeps(n):
        return -(-n // sweep) * sweep

    solver.reset()
    t_w = time.perf_counter()
    if sweep > 1 and a.steps % sweep:
        raise SystemExit(f"bench: the two-step sweep times whole sweeps: --steps must be even (got {a.steps})")
    if a.warmup > 0:
        solver.run_iterations(whole_sweeps(a.warmup), use_graph)
    solver.synchronize()
    # GPU clocks ramp up under load: a 20-step window that follows a short
    # warm-up or an idle gap ran 255-290 us per step, the same window after
    # 600 warm-up iterations 249 (tools/settle_probe.py, profiles/r4_settle.txt).
    # So the warm-up lasts at least --warmup-s seconds of sweeps (the same
    # extra count on every rank: the slowest rank's rate decides).
    # (counts are whole sweeps: the two-step sweep runs only even counts)
    clock_iters = 0
    n_w = whole_sweeps(a.warmup)
    if a.warmup_s > 0 and n_w == 0:  # (no warm-up steps asked for: time one sweep's worth to size the clock warm-up)
        n_w = whole_sweeps(2)
        solver.run_iterations(n_w, use_graph)
        solver.synchronize()
    dt_w = maxval(time.perf_counter() - t_w)
    if a.warmup_s > 0 and dt_w < a.warmup_s:
        per = dt_w / n_w
        clock_iters = min(20000, int((a.warmup_s - dt_w) / max(per, 1e-6)) + 1)
        clock_iters = whole_sweeps(int(maxval(float(clock_iters))))
        solver.run_iterations(clock_iters, use_graph)
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
                     t_check_s=maxval(tm.get("check", 0.0)),
                     t_breakdown_s={k: maxval(tm[k]) for k in ("gpu", "dot", "halo", "reduce", "wait", "copy")},
                     iters_converged=int(res.iters), converged=bool(res.converged),
                     l2_err=float(res.l2_err), max_err=float(res.max_err),
                     solve_iters_per_s=float(res.iters) / maxval(tm["iterate"]))
        if not a.no_random_solve:
            # BASELINE's "random-init w0": same solver, w0 = amp·hash(global
            # node, seed) (decomposition-independent); T_solver here has no
            # construction in it (counted once, by the first solve)
            solver.set_init(nat.Init.Random, a.seed, 0.05)
            barrier()
            rr = solver.solve()
            solver.set_init(nat.Init.Zero, a.seed, 0.05)
            extra["random_init"] = dict(seed=a.seed, amp=0.05, iters=int(rr.iters), converged=bool(rr.converged),
                                        t_solver_s=maxval(rr.timers["solver"]),
                                        t_iterate_s=maxval(rr.timers["iterate"]), l2_err=float(rr.l2_err),
                                        parity="unpinned vs reference (the reference has only w0 = 0)")

    ips = a.steps / dt
    pcis = sorted({r["pci_bus_id"] for r in ranks_info})
    out = {
        "metric": "pcg_iters_per_sec_8192x8192" if (M, N) == (8192, 8192) else f"pcg_iters_per_sec_{M}x{N}",
        "value": ips,
        "unit": "PCG iterations/s (global solve)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "clock_warmup_steps": clock_iters,
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
            "parallelism": f"2d-decomp {blk.Px}x{blk.Py} (halo: {solver.halo_path})" if world > 1 else "single-gpu",
            "points_per_s": ips * (M - 1) * (N - 1),
            "algo": (f"{['', '', 'two', 'three'][solver.sweep_steps]}-step sweep (1 kernel + 1 reduction per "
                     f"{solver.sweep_steps} iterations)" if solver.two_step else
                     "single-sweep (1 kernel, 1 allreduce / iter)" if solver.fused else
                     "classic (2 kernels, 2 allreduces / iter)"),
            "decomposition": {"spec": a.decomp, "Px": blk.Px, "Py": blk.Py, "block": [blk.nx, blk.ny]},
            "transport": comm.name if comm is not None else "none",
            "comm_ranks": comm.size if comm is not None else 1,
            "distinct_gpus": len(pcis),
            "ranks": ranks_info,
            "allreduce": ("in-sweep P2P over xGMI" if solver.xr else "launch per iteration") if world > 1 else "none",
            "halo": ("in-sweep xGMI push" + (" (graph-captured)" if use_graph and solver.graphs_usable else "")
                     if solver.halo_push else
                     "peer put over xGMI (kPut)" + (" (graph-captured)" if use_graph and solver.graphs_usable else "")
                     if solver.halo_put else
                     ("exchange: " + comm.name)) if world > 1 else "none",
            "overlap": bool(solver.overlap),
            # the construction's halo-path choice: every candidate's us per sweep (max over ranks; the two
            # fastest timed twice) and the pick
            "halo_path": solver.halo_path,
            "halo_candidates_us_per_sweep": [[n, round(us, 2)] for n, us in solver.halo_candidates],
            "exchange_us_measured": round(solver.exchange_us, 2),
            "item_order": "dynamic per-XCD queue" if solver.order == 3 else f"static {solver.layout_name} layout",
            "rows_per_item": solver.ti,
            # (a negative entry: another static layout tried at that height)
            "rows_per_item_candidates": list(solver.ti_tuning_rows),
            "rows_per_item_tuning_ms": [round(x, 4) for x in solver.ti_tuning_ms],
            "resident": bool(solver.resident),
            "chunk": solver.chunk,
            "launch": a.launch,
            "placement": {"candidates_ms_per_sweep": [round(x, 4) for x in solver.placement_ms],
                          "chosen": solver.placement_choice, "search_s": round(solver.placement_s, 3),
                          "job_ms_per_sweep": round(solver.placement_job_ms, 4)},
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

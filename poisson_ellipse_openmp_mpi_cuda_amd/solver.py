"""One entry point for every backend.

The reference ships five executables (stage0 serial, stage1 OpenMP, stage2
MPI, stage3 MPI+OpenMP, stage4 MPI+CUDA; README.md:7-13).  Here they are
backends of one solver:

==============  ==========================================================
backend         what runs
==============  ==========================================================
``serial``      native CPU oracle, 1 thread  (stage0; --norm unweighted = stage0's stop rule)
``omp``         native CPU, OpenMP threads   (stage1)
``ranks``       native CPU, P thread-ranks × T OpenMP threads (stage2 / stage3)
``dist-cpu``    one process per rank over torch.distributed gloo (stage2 / 3 multi-process)
``hip``         device-resident PCG on MI355X; one process per GPU over RCCL (stage4)
``hip-group``   P virtual ranks on one GPU (decomposition testing)
``torch``       PyTorch fp64 oracle (any torch device)
==============  ==========================================================
"""

from __future__ import annotations

import dataclasses
import time
from typing import Optional

import numpy as np

from ._loader import native
from .models.ellipse import EllipseProblem
from .parallel import decomp as _decomp

BACKENDS = ("serial", "omp", "ranks", "dist-cpu", "hip", "hip-group", "torch")


@dataclasses.dataclass
class SolveReport:
    backend: str
    M: int
    N: int
    ranks: int
    Px: int
    Py: int
    threads: int
    iters: int
    converged: bool
    breakdown: bool
    last_diff: float
    timers: dict
    l2_err: float
    max_err: float
    max_outside: float
    init: str = "zero"
    w: Optional[np.ndarray] = None
    rank: int = 0
    algo: str = ""
    nonfinite: bool = False
    history: Optional[list] = None  # ‖Δw‖ per iteration (keep_history=True)
    comm: str = ""  # device transport of a multi-rank HIP run (e.g. "rccl", "p2p-allreduce+rccl")
    xr: bool = False  # the sweep sums its scalars over ranks itself (P2P transport, no allreduce launch)
    halo_push: bool = False  # the sweep pushes its edge rows to the neighbours over xGMI (no exchange call)
    # first cross-device run diagnostics (this rank's): the P2P transport's set-up ("ok" / "fallback: why"),
    # the halo push's ("on" / "off: why" / "fallback: why"), the per-sweep sums' transport, and
    # hipDeviceCanAccessPeer toward every rank's device (1 / 0, -1 same device)
    overlap: bool = False  # the halo exchange runs on a second stream while the sweep's interior items run
    halo_put: bool = False  # the halo phases go through the peer-put kernel (p2p.hip kPut), not the comm
    # the halo path chosen at construction ("exchange" / "put" / "push" [+overlap]) and the candidates' timings
    # ([path, us per sweep], max over ranks), the peer put's set-up status
    halo_path: str = ""
    halo_candidates: Optional[list] = None
    put_status: str = ""
    p2p_sum_setup: str = ""
    push_status: str = ""
    sums: str = ""
    peer_access: Optional[list] = None
    resident_fallback: bool = False  # a resident launch aborted (barrier timeout); the solve finished streaming
    # end-of-solve true-residual check (device single-sweep-layout paths, -1: not computed): E-norm of
    # B - A w for the returned w, ||B||, and (three-step) the recurrence's ||r|| of the same iterate, the
    # gap ||B - A w - r|| / ||r||, and the restarts (residual replacement) the gap triggered
    res_true: float = -1.0
    res_rec: float = -1.0
    res_gap: float = -1.0
    b_norm: float = -1.0
    restarts: int = 0

    @property
    def iters_per_s(self) -> float:
        t = self.timers.get("iterate") or self.timers.get("solver") or 0.0
        return self.iters / t if t > 0 else 0.0

    def to_dict(self) -> dict:
        d = dataclasses.asdict(self)
        d.pop("w", None)
        d["iters_per_s"] = self.iters_per_s
        return d


ALGOS = {"auto": 0, "classic": 1, "fused": 2, "two-step": 3, "three-step": 4}


def _options(init="zero", seed=1234, threads=1, chunk=0, graph=False, timing=False, check_tol=True, variant=0,
             keep_history=False, log_every=0, algo="auto", checkpoint_every=0, checkpoint=None, resume=None):
    nat = native()
    o = nat.SolveOptions()
    o.init = nat.Init.Random if init == "random" else nat.Init.Zero
    o.seed = int(seed)
    o.threads = int(threads)
    o.chunk = int(chunk)
    o.use_graph = bool(graph)
    o.timing = bool(timing)
    o.check_tol = bool(check_tol)
    o.variant = int(variant)
    o.algo = ALGOS[algo] if isinstance(algo, str) else int(algo)
    o.keep_history = bool(keep_history)
    o.checkpoint_every = int(checkpoint_every)
    o.checkpoint_path = str(checkpoint or "")
    o.resume_path = str(resume or "")
    o.log_every = int(log_every)
    return o


def _report(backend, prob, res, ranks, threads, init, w=None, rank=0) -> SolveReport:
    return SolveReport(
        backend=backend, M=prob.M, N=prob.N, ranks=ranks, Px=res.Px, Py=res.Py, threads=threads,
        iters=int(res.iters), converged=bool(res.converged), breakdown=bool(res.breakdown),
        last_diff=float(res.last_diff), timers=dict(res.timers), l2_err=float(res.l2_err),
        max_err=float(res.max_err), max_outside=float(res.max_outside), init=init, w=w, rank=rank,
        algo=str(getattr(res, "algo", "")), nonfinite=bool(getattr(res, "nonfinite", False)),
        history=list(res.history) if len(res.history) else None,
        resident_fallback=bool(getattr(res, "resident_fallback", False)),
        res_true=float(getattr(res, "res_true", -1.0)), res_rec=float(getattr(res, "res_rec", -1.0)),
        res_gap=float(getattr(res, "res_gap", -1.0)),
        b_norm=float(getattr(res, "b_norm", -1.0)), restarts=int(getattr(res, "restarts", 0)))


def solve(prob: EllipseProblem, backend: str = "hip", ranks: int = 1, threads: int = 1, decomp: str | None = None,
          init: str = "zero", seed: int = 1234, return_w: bool = False, device: str = "cuda", **kw) -> SolveReport:
    """Solve the fictitious-domain Poisson problem with the chosen backend.

    For ``hip`` with torch.distributed initialised and world > 1 this is the
    per-rank call of a multi-GPU job (every rank calls it; rank 0's report
    carries the max-over-ranks timers and, with return_w, the gathered w).
    """
    if backend not in BACKENDS:
        raise ValueError(f"backend must be one of {BACKENDS}")
    decomp = decomp or _decomp.default_spec(backend)
    nat = native()
    P = prob.to_native()
    if backend in ("serial", "omp", "ranks"):
        t = 1 if backend == "serial" else max(1, threads)
        nranks = ranks if backend == "ranks" else 1
        opt = _options(init, seed, t, keep_history=kw.get("keep_history", False), log_every=kw.get("log_every", 0))
        res, w = nat.cpu_solve_grid(P, _decomp.grid(nranks, prob.M, prob.N, decomp if backend == "ranks" else "reference"),
                                    opt, return_w)
        return _report(backend, prob, res, nranks, t, init, None if w is None else np.asarray(w))
    if backend == "torch":
        import torch

        from .ops import torch_ref

        if device.startswith("cuda") and not torch.cuda.is_available():
            device = "cpu"
        t0 = time.perf_counter()
        r = torch_ref.pcg(prob, device=device, keep_history=kw.get("keep_history", False))
        dt = time.perf_counter() - t0
        timers = dict(solver=dt, iterate=dt)
        return SolveReport("torch", prob.M, prob.N, 1, 1, 1, 1, r.iters, r.converged, False,
                           r.history[-1] if r.history else 0.0, timers, r.l2_err, r.max_err, -1.0, "zero",
                           r.w[1:-1, 1:-1].cpu().numpy() if return_w else None)
    if backend == "hip-group":
        opt = _options(init, seed, chunk=kw.get("chunk", 0), timing=kw.get("timing", False),
                       variant=kw.get("variant", 0), check_tol=kw.get("check_tol", True),
                       algo=kw.get("algo", "auto"))
        res, w = nat.device_solve_group_grid(P, _decomp.grid(ranks, prob.M, prob.N, decomp), opt, return_w)
        return _report(backend, prob, res, ranks, 1, init, None if w is None else np.asarray(w))
    # distributed backends
    from .parallel import dist as _dist

    if backend == "dist-cpu":
        ctx = _dist.init()
        blk = _decomp.block(prob.M, prob.N, ctx.world, ctx.rank, decomp)
        opt = _options(init, seed, max(1, threads))
        res, w = nat.cpu_solve_rank(P, blk, *_dist.gloo_callbacks(), opt, True)
        wg = _dist.gather_blocks(ctx, prob, blk, np.asarray(w)) if return_w else None
        return _report(backend, prob, res, ctx.world, threads, init, wg, ctx.rank)
    # hip
    if nat.device_count() < 1:
        raise RuntimeError("backend 'hip' needs a visible MI355X (HIP device)")
    import torch.distributed as tdist

    if tdist.is_available() and tdist.is_initialized():
        world = tdist.get_world_size()
    else:
        world = _dist.env_rank_world()[1]
    opt = _options(init, seed, chunk=kw.get("chunk", 0), graph=kw.get("graph", False), timing=kw.get("timing", False),
                   check_tol=kw.get("check_tol", True), variant=kw.get("variant", 0), algo=kw.get("algo", "auto"),
                   checkpoint_every=kw.get("checkpoint_every", 0), checkpoint=kw.get("checkpoint"),
                   resume=kw.get("resume"), keep_history=kw.get("keep_history", False),
                   log_every=kw.get("log_every", 0))
    if world == 1:
        rank, comm = 0, None
        nat.set_device(0)
        blk = _decomp.block(prob.M, prob.N, 1, 0, decomp)
    else:
        ctx = _dist.init()
        rank = ctx.rank
        comm = _dist.rccl_comm(ctx)
        blk = _decomp.block(prob.M, prob.N, world, rank, decomp)
    solver = nat.DeviceSolver(P, blk, comm, opt)
    try:
        res = solver.solve()
    except Exception:
        if comm is not None:
            _dist.drop_comm(comm)
        raise
    if comm is not None and (res.nonfinite or not np.isfinite(res.last_diff)):
        _dist.drop_comm(comm)  # its P2P sequence may be out of step with the peers'
    w = None
    if return_w:
        wl = np.asarray(solver.w())
        if world == 1:
            w = wl
        else:
            w = _dist.gather_blocks(_dist.init(), prob, blk, wl)
    rep = _report("hip", prob, res, world, 1, init, w, rank)
    rep.comm = comm.name if comm is not None else "self"
    rep.xr = bool(solver.xr)
    rep.halo_push = bool(solver.halo_push)
    rep.overlap = bool(solver.overlap)
    rep.halo_put = bool(solver.halo_put)
    rep.halo_path = str(solver.halo_path)
    rep.halo_candidates = [[str(n), round(float(us), 2)] for n, us in solver.halo_candidates]
    rep.put_status = str(solver.put_status)
    rep.p2p_sum_setup = str(nat.p2p_setup_status())
    rep.push_status = str(solver.push_status)
    rep.sums = str(solver.xr_status)
    rep.peer_access = [int(v) for v in solver.peer_access]
    return rep

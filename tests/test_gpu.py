"""MI355X tests: the gfx950 kernels and the device-resident solver.

Numerics are checked against the CPU oracle (native serial backend, itself
bit-compatible with the reference) and the PyTorch fp64 oracle; iteration
counts against the published / survey golden values.  Every test runs the
native HIP path (the extension fails loudly when missing)."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve
from poisson_ellipse_openmp_mpi_cuda_amd.models.ellipse import GOLDEN_ITERS, GOLDEN_L2
from poisson_ellipse_openmp_mpi_cuda_amd.ops import device as dops
from poisson_ellipse_openmp_mpi_cuda_amd.ops import torch_ref
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("M,N,norm", [(40, 40, "weighted"), (40, 40, "unweighted"), (400, 600, "weighted"),
                                      (800, 1200, "weighted"), (2048, 2048, "weighted"), (10, 10, "unweighted")])
@pytest.mark.parametrize("variant,algo", [(0, "fused"), (0, "classic"), (1, "classic")])
def test_device_golden_iterations(gpu, M, N, norm, variant, algo):
    rep = solve(EllipseProblem(M, N, norm=norm), backend="hip", variant=variant, algo=algo)
    assert rep.converged
    assert rep.iters == GOLDEN_ITERS[(M, N, norm)]
    if (M, N) in GOLDEN_L2 and norm == "weighted":
        assert rep.l2_err == pytest.approx(GOLDEN_L2[(M, N)], rel=5e-3)


@pytest.mark.parametrize("M,N", [(40, 40), (257, 129), (400, 600)])
def test_device_solution_matches_cpu_oracle(gpu, M, N):
    prob = EllipseProblem(M, N)
    ref = solve(prob, backend="serial", return_w=True)
    for variant, algo in ((0, "fused"), (0, "classic"), (1, "classic")):
        rep = solve(prob, backend="hip", return_w=True, variant=variant, algo=algo)
        assert rep.iters == ref.iters
        np.testing.assert_allclose(rep.w, ref.w, rtol=0, atol=1e-10)


@pytest.mark.parametrize("ranks,decomp", [(2, "aspect"), (3, "aspect"), (4, "aspect"), (6, "aspect"),
                                          (8, "reference"), (5, "aspect"), (4, "rows"), (6, "2x3"), (3, "cols")])
@pytest.mark.parametrize("algo", ["fused", "classic"])
def test_virtual_ranks_match_single(gpu, ranks, decomp, algo):
    prob = EllipseProblem(300, 420)
    one = solve(prob, backend="hip", return_w=True, algo=algo)
    grp = solve(prob, backend="hip-group", ranks=ranks, decomp=decomp, return_w=True, algo=algo)
    assert grp.Px * grp.Py == ranks
    assert abs(grp.iters - one.iters) <= 1
    np.testing.assert_allclose(grp.w, one.w, rtol=0, atol=1e-9)
    assert grp.l2_err == pytest.approx(one.l2_err, rel=1e-6)


@pytest.mark.parametrize("M,N,ranks,decomp", [(7, 7, 9, "aspect"), (9, 5, 4, "aspect"), (25, 13, 12, "aspect"),
                                               (9, 9, 16, "aspect")])
def test_fused_thin_blocks(gpu, M, N, ranks, decomp):
    # blocks down to 2 rows / columns (3x3 of 2x2 blocks: every halo node and
    # corner comes from a neighbour); 8x2 of 1-row blocks falls back to classic
    prob = EllipseProblem(M, N)
    one = solve(prob, backend="hip", return_w=True, algo="classic")
    grp = solve(prob, backend="hip-group", ranks=ranks, decomp=decomp, return_w=True)
    assert abs(grp.iters - one.iters) <= 1
    np.testing.assert_allclose(grp.w, one.w, rtol=0, atol=1e-9)


@pytest.mark.parametrize("M,N", [(4096, 4096), (8192, 8192), (16384, 16384)])
def test_fused_large_golden(gpu, M, N):
    rep = solve(EllipseProblem(M, N), backend="hip", algo="fused")
    assert rep.converged and rep.iters == GOLDEN_ITERS[(M, N, "weighted")]
    assert rep.l2_err == pytest.approx(GOLDEN_L2[(M, N)], rel=5e-3)


@pytest.mark.parametrize("iters", [40, 41])
def test_fused_matches_classic_state(gpu, nat, iters):
    # odd counts end on a deferring sweep: w() must flush the pending α·p term
    prob = EllipseProblem(300, 500)
    blk = D.block(300, 500, 1, 0)
    out = {}
    for algo in (1, 2):
        opt = nat.SolveOptions()
        opt.algo = algo
        opt.check_tol = False
        s = nat.DeviceSolver(prob.to_native(), blk, None, opt)
        assert s.fused == (algo == 2)
        s.reset()
        s.run_iterations(iters, False)
        s.synchronize()
        out[algo] = (s.state(), s.w())
    (sc, wc), (sf, wf) = out[1], out[2]
    assert sc["iter"] == sf["iter"] == iters
    assert sf["alpha"] == pytest.approx(sc["alpha"], rel=1e-9)
    assert sf["beta"] == pytest.approx(sc["beta"], rel=1e-9)
    np.testing.assert_allclose(wf, wc, rtol=0, atol=1e-12 * np.abs(wc).max())


@pytest.mark.parametrize("algo", [1, 2])
def test_run_iterations_parity_across_calls(gpu, nat, algo):
    # 3 + 4 + 5 iterations (graph and eager, odd boundaries) == 12 in one call
    prob = EllipseProblem(200, 260)
    blk = D.block(200, 260, 1, 0)
    res = []
    for parts in ([12], [3, 4, 5]):
        opt = nat.SolveOptions()
        opt.algo = algo
        opt.check_tol = False
        opt.chunk = 4
        s = nat.DeviceSolver(prob.to_native(), blk, None, opt)
        s.reset()
        for n in parts:
            s.run_iterations(n, True)
        s.synchronize()
        res.append((s.state()["iter"], s.w()))
    assert res[0][0] == res[1][0] == 12
    assert np.array_equal(res[0][1], res[1][1])


@pytest.mark.parametrize("M,N", [(40, 40), (400, 600), (10, 10)])
def test_fused_odd_convergence_and_cap(gpu, M, N):
    # convergence on a deferring (odd) sweep and an odd iteration cap both
    # leave a complete w
    prob = EllipseProblem(M, N)
    a = solve(prob, backend="hip", return_w=True, algo="classic")
    b = solve(prob, backend="hip", return_w=True, algo="fused")
    assert a.iters == b.iters
    np.testing.assert_allclose(b.w, a.w, rtol=0, atol=1e-10)
    capped = EllipseProblem(M, N)
    capped.max_iter = 7
    c = solve(capped, backend="hip", return_w=True, algo="classic")
    d = solve(capped, backend="hip", return_w=True, algo="fused")
    assert c.iters == d.iters == 7 and not d.converged
    np.testing.assert_allclose(d.w, c.w, rtol=0, atol=1e-9 * max(1e-30, np.abs(c.w).max()))


@pytest.mark.parametrize("order", ["0", "2", "3"])
def test_fused_item_orders_deterministic(gpu, order, monkeypatch):
    # order 3 = per-XCD dynamic work queue: which wave takes which item varies
    # run to run, the per-item sums keep the result bitwise reproducible
    monkeypatch.setenv("PE_ORDER", order)
    monkeypatch.setenv("PE_RESIDENT", "0")  # the streaming sweep (800×1200 would run resident)
    prob = EllipseProblem(800, 1200)
    a = solve(prob, backend="hip", return_w=True, algo="fused")
    b = solve(prob, backend="hip", return_w=True, algo="fused")
    assert a.iters == b.iters == 989
    assert np.array_equal(a.w, b.w)
    monkeypatch.setenv("PE_ORDER", "0")
    c = solve(prob, backend="hip", return_w=True, algo="fused")
    np.testing.assert_allclose(a.w, c.w, rtol=0, atol=1e-10)


def test_virtual_ranks_golden_grid(gpu):
    rep = solve(EllipseProblem(1600, 2400), backend="hip-group", ranks=4)
    assert rep.iters == GOLDEN_ITERS[(1600, 2400, "weighted")]


@pytest.mark.parametrize("M,N,kw", [(40, 40, {}), (257, 129, {}), (600, 400, {}),
                                    (512, 512, dict(A2=-1.0, B2=1.0, cy=1.0)),
                                    (300, 200, dict(A1=-2.0, B1=2.0, A2=-1.0, B2=1.0, cx=0.25, cy=1.0))])
def test_device_operator_vs_torch_oracle(gpu, M, N, kw):
    prob = EllipseProblem(M, N, **kw)
    a, b, _ = torch_ref.assemble(prob, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(1)
    p = torch.rand(M + 1, N + 1, dtype=torch.float64, device="cuda", generator=g) - 0.5
    p[0, :] = p[-1, :] = 0
    p[:, 0] = p[:, -1] = 0
    ref = torch_ref.apply_A(p, a, b, prob.h1, prob.h2).cpu().numpy()
    got = dops.apply_A_device(prob, p.cpu().numpy())
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() <= 1e-13 * scale
    # coefficients seen by the kernels == reference assembly, bitwise
    ad, bd, Dd = dops.coefficients_device(prob)
    at, bt = a.cpu().numpy(), b.cpu().numpy()
    assert np.array_equal(ad, at)
    assert np.array_equal(bd, bt)
    Dt = torch_ref.diag(a, b, prob.h1, prob.h2).cpu().numpy()
    np.testing.assert_array_equal(Dd[1:M, 1:N], Dt[1:M, 1:N])


def test_random_init_matches_cpu(gpu):
    prob = EllipseProblem(200, 300)
    c = solve(prob, backend="serial", init="random", seed=11, return_w=True)
    d = solve(prob, backend="hip", init="random", seed=11, return_w=True)
    assert abs(c.iters - d.iters) <= 1
    np.testing.assert_allclose(d.w, c.w, rtol=0, atol=1e-9)


def test_bitwise_deterministic_and_graph_equivalent(gpu, monkeypatch):
    monkeypatch.setenv("PE_RESIDENT", "0")  # the streaming sweep (500×700 would run resident)
    prob = EllipseProblem(500, 700)
    a = solve(prob, backend="hip", return_w=True, algo="fused")  # eager launches (default)
    b = solve(prob, backend="hip", return_w=True, algo="fused")
    c = solve(prob, backend="hip", return_w=True, graph=True, algo="fused")  # chunks replayed from hipGraphs
    assert a.iters == b.iters == c.iters
    assert np.array_equal(a.w, b.w) and np.array_equal(a.w, c.w)


def test_timing_mode_breakdown(gpu):
    rep = solve(EllipseProblem(800, 1200), backend="hip", timing=True)
    assert rep.iters == 989
    t = rep.timers
    assert t["gpu"] > 0 and t["solver"] >= t["gpu"] * 0.5


def test_fixed_iterations_no_tol(gpu, nat):
    prob = EllipseProblem(400, 600)
    blk = D.block(400, 600, 1, 0)
    opt = nat.SolveOptions()
    opt.check_tol = False
    s = nat.DeviceSolver(prob.to_native(), blk, None, opt)
    s.reset()
    s.run_iterations(700, True)
    s.synchronize()
    st = s.state()
    assert st["iter"] == 700 and st["status"] == 0 and st["done"] == 0
    dt = s.time_iterations(100, True)
    assert dt > 0 and s.state()["iter"] == 800


def test_rccl_single_rank_comm(gpu, nat):
    uid = nat.rccl_unique_id()
    assert isinstance(uid, bytes) and len(uid) == 128
    comm = nat.make_rccl_comm(uid, 0, 1)
    assert comm.size == 1 and comm.name == "rccl"
    prob = EllipseProblem(400, 600)
    s = nat.DeviceSolver(prob.to_native(), D.block(400, 600, 1, 0), comm, nat.SolveOptions())
    r = s.solve()
    assert r.iters == 546


def test_native_apps(gpu):
    exe = os.path.join(ROOT, "bin", "pe_hip")
    out = subprocess.run([exe, "800", "1200"], capture_output=True, text=True, check=True, timeout=120).stdout
    assert "M=800, N=1200 | Iter=989 | Total Time=" in out
    assert "GPU compute time (Ap + D^{-1}r, max over ranks)" in out
    out = subprocess.run([os.path.join(ROOT, "bin", "pe_launch"), "-n", "1", exe, "--json", "400", "600"],
                         capture_output=True, text=True, check=True, timeout=120).stdout
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert d["iters"] == 546
    out = subprocess.run([exe, "--vranks", "4", "--json", "400", "600"], capture_output=True, text=True, check=True,
                         timeout=120).stdout
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert d["iters"] == 546 and d["ranks"] == 4


def test_bench_contract(gpu):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "50", "--warmup", "5", "--grid",
                          "1024", "1024"], capture_output=True, text=True, check=True, timeout=300).stdout
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["steps"] == 50 and d["n_gpus"] == 1 and d["valid"] and d["value"] > 0
    assert d["converged"] and d["l2_err"] < 1e-3


@pytest.mark.parametrize("warmup", ["0", "5"])
def test_bench_two_step_warmup_counts(gpu, warmup):
    """The clock warm-up and an odd --warmup run whole two-step sweeps (an odd
    count used to make run_iterations throw)."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--algo", "two-step", "--steps", "10",
                          "--warmup", warmup, "--warmup-s", "0.05", "--no-solve", "--grid", "512", "512"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["valid"] and d["steps"] == 10 and d["clock_warmup_steps"] % 2 == 0


def test_graft_smoke(gpu):
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g

    g.smoke()


def test_two_process_device_path_host_staged(gpu):
    """torchrun-style 2-process job on the one GPU: torch.distributed bootstrap,
    per-rank blocks, halo plan, timer reduction and gather — with the
    host-staged transport (RCCL refuses two ranks on one device)."""
    from conftest import free_port

    env = dict(os.environ, PE_COMM="host")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "poisson_ellipse_openmp_mpi_cuda_amd", "--json",
           "--quiet", "400", "600"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["iters"] == 546 and d["ranks"] == 2 and d["Px"] * d["Py"] == 2
    assert d["l2_err"] == pytest.approx(3.06e-4, rel=5e-3)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "30", "--warmup", "3", "--grid", "512", "512"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["valid"] and d["converged"]


def test_halo_choice_agrees_when_ranks_tune_differently(gpu):
    """Each rank tunes its own rows per item — or not at all past 2²⁵ nodes —
    so the overlap's candidate heights can differ in number between ranks;
    the halo-path choice agrees on one count first (every rank then times as
    many candidates and calls the cross-rank max as often).  8194×8192 on 2
    row slabs: rank 0's block is 4096×8191 (tuned: three heights), rank 1's
    4097×8191 (2²⁵ nodes and more: not tuned, one height).  Before the
    agreement the job hung in the choice's collectives.  Host-staged transport,
    P2P sums (the put candidates too), 30 iterations."""
    from conftest import free_port

    base = {k: v for k, v in os.environ.items() if k not in ("PE_HALO", "PE_OVERLAP", "PE_STEPS", "PE_TI", "PE_TI_TUNE")}
    env = dict(base, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60", PE_XR="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
           "poisson_ellipse_openmp_mpi_cuda_amd", "--json", "--quiet", "--decomp", "rows", "--max-iter", "30",
           "8194", "8192"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["ranks"] == 2 and d["iters"] == 30
    names = [n for n, _ in d["halo_candidates"] if "(again)" not in n]
    assert sum(1 for n in names if n.startswith("exchange+overlap")) == 1, names  # (the agreed count: rank 1's one)
    assert "exchange" in names and "put" in names, names


@pytest.mark.parametrize("nproc,decomp,allreduce,env", [
    # the default path (no PE_HALO / PE_OVERLAP): chosen at construction by timing
    (4, "aspect", "p2p", {}), (3, "rows", "p2p", {}), (4, "rows", "p2p", {}), (2, "aspect", "p2p", {}),
    (4, "aspect", "rccl", {}),
    # each path forced: the comm's exchange with the overlap on the default slabs
    # (kSignal on a row slab, the multi-GPU default since round 5), the peer put
    # (IPC-mapped inboxes of the other processes), the sweep's push
    (3, "rows", "p2p", {"PE_HALO": "exchange", "PE_OVERLAP": "1"}),
    (4, "rows", "p2p", {"PE_HALO": "put", "PE_OVERLAP": "1"}), (4, "aspect", "p2p", {"PE_HALO": "put"}),
    (3, "rows", "p2p", {"PE_HALO": "push"}),
    (3, "aspect", "rccl", {"PE_OVERLAP": "1"}), (4, "aspect", "p2p-kernel", {"PE_OVERLAP": "1"}),
    # the single sweep and its overlap
    (4, "aspect", "rccl", {"PE_OVERLAP": "1", "PE_STEPS": "1"}),
])
def test_multi_process_2d_host_staged(gpu, nproc, decomp, allreduce, env):
    """3-4 processes on the one GPU, 2×2 blocks (y-strip phase, unpack, corner
    rows through the x phase) and 3×1 / 4×1 row slabs, match the
    single-process solution (gathered w).  The halo path is the construction's
    choice — timed on this job's transport — or forced: the host-staged
    transport's exchange (with the boundary / interior overlap on two
    streams), the peer-put kernel through the other processes' IPC-mapped
    inboxes, or the sweep's own push.  The per-iteration sums go through the
    host-staged transport ("rccl"), the P2P transport summed inside the
    sweep's final reduction block ("p2p"), or the standalone one-shot P2P
    kernel ("p2p-kernel", PE_XR=0)."""
    from conftest import free_port

    tag = "_".join(f"{k}{v}" for k, v in sorted(env.items()))
    base = {k: v for k, v in os.environ.items() if k not in ("PE_HALO", "PE_OVERLAP", "PE_STEPS")}
    env = dict(base, PE_COMM="host", PE_ALLREDUCE=allreduce.split("-")[0], PE_P2P_TIMEOUT_S="60",
               PE_XR="0" if allreduce == "p2p-kernel" else "1", **env)
    outp = os.path.join(ROOT, "gpurun_out", f"mp_w_{nproc}_{decomp}_{allreduce}_{tag}.npy")
    os.makedirs(os.path.dirname(outp), exist_ok=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
           "poisson_ellipse_openmp_mpi_cuda_amd", "--json", "--quiet", "--decomp", decomp, "--dump", outp, "300", "420"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["ranks"] == nproc and d["Px"] * d["Py"] == nproc
    assert d["comm"] == ("p2p-allreduce+host-staged" if allreduce.startswith("p2p") else "host-staged")
    assert d["xr"] == (allreduce == "p2p")
    path = d["halo_path"]
    assert d["halo_push"] == path.startswith("push") and d["halo_put"] == path.startswith("put"), d
    assert d["overlap"] == ("+overlap" in path), path
    if "PE_HALO" in env:
        assert path.startswith(env["PE_HALO"]), path
    if "PE_OVERLAP" in env:
        assert d["overlap"] == (env["PE_OVERLAP"] == "1"), path
    if not allreduce.startswith("p2p"):  # no IPC-mapped transport: the exchange only
        assert path.startswith("exchange"), path
    elif "PE_HALO" not in env and "PE_OVERLAP" not in env:
        names = [n for n, _ in d["halo_candidates"]]
        assert "put" in names and "exchange" in names and ("push" in names) == (d["Py"] == 1 and d["xr"]), names
    assert d["algo"] == ("fused" if env.get("PE_STEPS") == "1" else "three-step"), d["algo"]
    one = solve(EllipseProblem(300, 420), backend="hip", return_w=True)
    assert abs(d["iters"] - one.iters) <= 1
    w = np.load(outp)
    np.testing.assert_allclose(w, one.w, rtol=0, atol=1e-9)


@pytest.mark.parametrize("nproc,decomp,allreduce,overlap", [(2, "1x2", "p2p", "0"), (4, "2x2", "rccl", "0"),
                                                             (6, "2x3", "p2p", "0"), (4, "2x2", "p2p", "1"),
                                                             (2, "1x2", "rccl", "1"), (6, "2x3", "p2p", "1")])
def test_multi_process_2d_three_step(gpu, nproc, decomp, allreduce, overlap):
    """2-D splits run the three-step sweep through the exchange: 6 columns of
    r and p per owned row packed after each sweep (kPack), exchanged and
    unpacked, then the x rows with their halo columns (the corners come from
    the diagonal rank).  300×437: every block's last strip has output lanes
    past ny, i.e. in the UP neighbour's columns, which the lane-tested march
    keeps out of the sums (item_layout never flags those items uniform).
    Iteration count and gathered w match one process.  PE_OVERLAP=1: the
    boundary items (the 6 owned rows / columns next to a neighbour) run first
    and count themselves (kS3's kSignal variant); pack + exchange + unpack run
    on the halo stream while the interior items are computed."""
    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE=allreduce, PE_P2P_TIMEOUT_S="60", PE_OVERLAP=overlap)
    outp = os.path.join(ROOT, "gpurun_out", f"mp3_w_{nproc}_{decomp}_{overlap}.npy")
    os.makedirs(os.path.dirname(outp), exist_ok=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
           "poisson_ellipse_openmp_mpi_cuda_amd", "--json", "--quiet", "--decomp", decomp, "--dump", outp, "300", "437"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["ranks"] == nproc and d["Py"] > 1 and d["algo"] == "three-step", d
    assert not d["halo_push"] and d["overlap"] == (overlap == "1")
    one = solve(EllipseProblem(300, 437), backend="hip", return_w=True)
    assert abs(d["iters"] - one.iters) <= 1
    np.testing.assert_allclose(np.load(outp), one.w, rtol=0, atol=1e-9)


def test_halo_push_selftest_failure_falls_back(gpu):
    """A failed halo-push self-test on ONE rank (PE_FAULT_INJECT=pushtest@rank:1)
    makes every rank keep the exchange: the job still solves correctly."""
    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60", PE_HALO="push",
               PE_FAULT_INJECT="pushtest@rank:1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "poisson_ellipse_openmp_mpi_cuda_amd", "--json",
           "--quiet", "--decomp", "rows", "400", "600"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["ranks"] == 3 and d["Py"] == 1 and d["xr"] and not d["halo_push"]
    assert d["iters"] == 546
    assert "halo push unavailable" in out.stderr
    # rank 0's own diagnostics say why (the failure was rank 1's)
    assert d["push_status"] == "fallback: self-test failed on a peer" and d["p2p_sum_setup"] == "ok"
    assert d["sums"] == "in-sweep P2P over xGMI"


def test_halo_put_selftest_failure_falls_back(gpu):
    """A failed peer-put self-test on ONE rank (PE_FAULT_INJECT=puttest@rank:1)
    takes the put out of every rank's candidates; the job solves correctly on
    the path chosen among the rest."""
    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60",
               PE_FAULT_INJECT="puttest@rank:1")
    env.pop("PE_HALO", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "poisson_ellipse_openmp_mpi_cuda_amd", "--json",
           "--quiet", "--decomp", "rows", "400", "600"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert "halo put unavailable" in out.stderr
    assert d["put_status"] == "fallback: self-test failed on a peer" and not d["halo_put"]
    names = [n for n, _ in d["halo_candidates"]]
    assert not any(n.startswith("put") for n in names) and "push" in names, names
    assert d["iters"] == 546


def test_halo_put_checkpoint_resume_bitwise(gpu, tmp_path):
    """Row slabs exchanging through the peer put (3 processes, IPC-mapped
    inboxes): a checkpointed and resumed job ends bitwise where the
    uninterrupted one does (the put keeps no halo state of its own: its
    counters restart with the new solvers on every rank)."""
    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60", PE_HALO="put")
    ck = str(tmp_path / "ck")

    def run(*extra):
        outp = str(tmp_path / f"w{len(extra)}.npy")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
               "127.0.0.1", "--master-port", str(free_port()), "-m", "poisson_ellipse_openmp_mpi_cuda_amd", "--json",
               "--quiet", "--decomp", "rows", "--dump", outp, *extra, "400", "600"]
        out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-3000:]
        d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
        assert d["halo_put"] and d["halo_path"].startswith("put"), d["halo_path"]
        return d, np.load(outp)

    full, wf = run("--checkpoint", ck, "--checkpoint-every", "200")
    assert full["iters"] == 546 and os.path.exists(ck + ".r2")
    res, wr = run("--resume", ck)
    assert res["iters"] == full["iters"]
    assert np.array_equal(wr, wf)


def test_p2p_selftest_failure_falls_back(gpu):
    """A failed P2P-sum self-test on ONE rank (PE_FAULT_INJECT=p2ptest@rank:1):
    every rank keeps the base transport for the sums (so no in-sweep sum and
    no halo push); the labels say why, and the job solves correctly."""
    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60",
               PE_FAULT_INJECT="p2ptest@rank:1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "-m", "poisson_ellipse_openmp_mpi_cuda_amd", "--json",
           "--quiet", "--decomp", "rows", "400", "600"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["ranks"] == 3 and not d["xr"] and not d["halo_push"] and d["comm"] == "host-staged"
    assert d["p2p_sum_setup"] == "fallback: self-test sum wrong on a peer"
    assert d["push_status"].startswith("off: no P2P transport") and d["sums"].startswith("allreduce launch")
    assert d["put_status"].startswith("off: no P2P transport") and d["halo_path"].startswith("exchange")
    assert d["peer_access"] == [-1, -1, -1]  # one GPU shared by the ranks
    assert d["iters"] == 546


def test_halo_push_checkpoint_resume_bitwise(gpu, tmp_path):
    """Row slabs with the halo push keep their halo rows in the receive
    buffers (the sweeps read them there): a checkpoint imports them into x
    first, a resume seeds the receive buffer from x — the resumed 3-rank job
    ends bitwise where the uninterrupted one does."""
    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60", PE_HALO="push")
    ck = str(tmp_path / "ck")

    def run(*extra):
        outp = str(tmp_path / f"w{len(extra)}.npy")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
               "127.0.0.1", "--master-port", str(free_port()), "-m", "poisson_ellipse_openmp_mpi_cuda_amd", "--json",
               "--quiet", "--decomp", "rows", "--dump", outp, *extra, "400", "600"]
        out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-3000:]
        d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
        assert d["halo_push"]
        return d, np.load(outp)

    full, wf = run("--checkpoint", ck, "--checkpoint-every", "200")
    assert full["iters"] == 546 and os.path.exists(ck + ".r2")
    res, wr = run("--resume", ck)
    assert res["iters"] == full["iters"]
    assert np.array_equal(wr, wf)


@pytest.mark.parametrize("nproc,halo", [(2, "push"), (4, "push"), (3, "put")])
def test_bench_halo_push_graphs(gpu, nproc, halo):
    """bench.py on row slabs over the P2P transport (processes sharing the
    one GPU, host-staged base transport for set-up only): the sweep pushes its
    edge rows into the neighbours' IPC-mapped receive buffers (the in-sweep
    sum's flags deliver them), or the peer-put kernel exchanges them through
    the neighbours' inboxes — no comm call in the iteration either way, so the
    iterations run as captured hipGraphs: the timed steps are valid and the
    full solve converges in the single-GPU iteration count."""
    from conftest import free_port

    M = N = 1024
    one = solve(EllipseProblem(M, N), backend="hip")
    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60", PE_HALO=halo, PE_OVERLAP="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--steps", "40", "--warmup", "4", "--grid", str(M), str(N), "--decomp", "rows",
           "--launch", "graph"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    c = d["config"]
    assert c["decomposition"]["Px"] == nproc and c["decomposition"]["Py"] == 1
    assert c["halo"] == ("in-sweep xGMI push" if halo == "push" else "peer put over xGMI (kPut)") + " (graph-captured)", c
    assert c["halo_path"].startswith(halo)
    assert c["allreduce"] == "in-sweep P2P over xGMI"
    assert c["algo"].startswith("three-step")
    assert d["valid"] and d["converged"] and abs(d["iters_converged"] - one.iters) <= 1
    assert d["l2_err"] == pytest.approx(one.l2_err, rel=1e-6)


@pytest.mark.parametrize("fault", ["pushtest@rank:1", "p2ptest@rank:1"])
def test_bench_reports_transport_fallbacks(gpu, fault):
    """A first cross-device run must say why it fell back:
    with one rank's halo-push or P2P-sum self-test failing, bench still
    succeeds (rc 0: a clean fallback) and every rank's entry in its JSON names
    the set-up outcome and the transport the sweep finally uses."""
    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60", PE_HALO="push", PE_FAULT_INJECT=fault)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "3", "--steps", "12", "--warmup", "3", "--grid", "400", "600", "--decomp", "rows",
           "--no-random-solve"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    ranks = d["config"]["ranks"]
    assert len(ranks) == 3 and d["valid"] and d["converged"] and d["iters_converged"] == 546
    for r in ranks:
        assert set(r["neighbors"]) == ({"right"} if r["rank"] == 0 else {"left"} if r["rank"] == 2 else {"left", "right"})
        assert all(v == -1 for v in r["peer_access"].values())  # the ranks share one GPU
        if fault.startswith("pushtest"):
            assert r["p2p_sum_setup"] == "ok" and r["sums"] == "in-sweep P2P over xGMI"
            assert r["halo_push"] == ("fallback: self-test failed on this rank" if r["rank"] == 1
                                      else "fallback: self-test failed on a peer")
        else:
            assert r["p2p_sum_setup"] == ("fallback: self-test sum wrong on this rank" if r["rank"] == 1
                                          else "fallback: self-test sum wrong on a peer")
            assert r["halo_push"].startswith("off: no P2P transport") and r["sums"].startswith("allreduce launch")
    assert d["config"]["halo"].startswith("exchange")


def test_bench_self_launch_and_random_init(gpu):
    """`bench.py --gpus 2` with no launcher starts its 2 ranks itself (here
    sharing the one GPU through the host-staged test transport): one JSON
    line, n_gpus 2, every rank listed with its device, the job-wide placement
    and the random-init solve reported."""
    env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "20",
                          "--warmup", "2", "--grid", "512", "512", "--decomp", "rows"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    c = d["config"]
    assert d["n_gpus"] == 2 and c["comm_ranks"] == 2 and d["valid"] and d["converged"]
    assert [r["rank"] for r in c["ranks"]] == [0, 1] and all(r["pci_bus_id"] for r in c["ranks"])
    ri = d["random_init"]
    assert ri["converged"] and ri["iters"] > 0 and ri["l2_err"] < 1e-2
    assert "wait" in d["t_breakdown_s"]


def test_bench_stalled_rank_fails_fast(gpu):
    """bench.py under torchrun with rank 1 stalled (PE_FAULT_INJECT=stall@rank:1):
    its bounded wait (PE_WATCHDOG_S) fires, the rank exits non-zero and the
    job ends — within 90 s, never a hang."""
    import signal

    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_FAULT_INJECT="stall@rank:1", PE_WATCHDOG_S="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "20", "--warmup", "2", "--grid", "512", "512"]
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=90)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        pytest.fail("a stalled rank hung bench.py instead of failing it")
    assert p.returncode != 0
    assert "watchdog" in err, err[-3000:]


def test_slow_rank_shows_in_tmpi(gpu):
    """T_MPI of the default multi-rank path (in-sweep P2P sums + halo push):
    with rank 1's sweeps idling 300 µs before their cross-rank sum
    (PE_FAULT_INJECT=slow@rank:1,us:300) the job's `wait` timer — max over
    ranks, rank 0 waits for rank 1 every iteration — is ≈ iterations × 300 µs
    (reference T_MPI: poisson_mpi_cuda2.cu:870-873, :891-895, :924-928, max over
    ranks :962-966)."""
    from conftest import free_port

    def run(fault):
        env = dict(os.environ, PE_COMM="host", PE_ALLREDUCE="p2p", PE_P2P_TIMEOUT_S="60", PE_HALO="push")
        if fault:
            env["PE_FAULT_INJECT"] = fault
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
               "poisson_ellipse_openmp_mpi_cuda_amd", "--json", "--quiet", "--decomp", "rows", "400", "600"]
        out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-3000:]
        d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
        assert d["xr"] and d["iters"] == 546
        return d["timers"]["wait"], d["algo"]

    base, algo = run(None)
    slow, _ = run("slow@rank:1,us:300")
    sums = 546 // {"three-step": 3, "two-step": 2}.get(algo, 1)  # one cross-rank sum per sweep
    want = sums * 300e-6
    assert 0.7 * want <= slow - base <= 2.0 * want, (base, slow, algo)


@pytest.mark.parametrize("algo", ["fused", "classic"])
def test_fault_injection_nan_stops_cleanly(gpu, algo, monkeypatch):
    monkeypatch.setenv("PE_FAULT_INJECT", "nan@iter:20")
    rep = solve(EllipseProblem(400, 600), backend="hip", algo=algo)
    assert rep.nonfinite and not rep.converged
    assert 20 <= rep.iters <= 23


@pytest.mark.parametrize("K", [20, 21])
def test_forced_breakdown_terminal_path(gpu, K, monkeypatch):
    """|den| < 1e-15 (PE_FAULT_INJECT=zero@iter:K zeroes the (p, A p) sums of
    sweep K) stops the solve at iteration K+1 before its update (reference
    :413) — K = 20: the breakdown is met by a deferring sweep (nothing
    pending), K = 21: by an applying sweep (it adds the pending α_K p_K).
    Every wave takes the terminal path (wave-counted hand-off, no workgroup
    barrier); w equals a run capped at K iterations."""
    prob = EllipseProblem(200, 300)
    monkeypatch.setenv("PE_RESIDENT", "0")
    monkeypatch.setenv("PE_FAULT_INJECT", f"zero@iter:{K}")
    brk = solve(prob, backend="hip", return_w=True, algo="fused")
    assert brk.breakdown and not brk.converged and brk.iters == K + 1
    monkeypatch.delenv("PE_FAULT_INJECT")
    capped = EllipseProblem(200, 300)
    capped.max_iter = K
    ref = solve(capped, backend="hip", return_w=True, algo="fused")
    assert ref.iters == K
    np.testing.assert_allclose(brk.w, ref.w, rtol=0, atol=1e-15 * np.abs(ref.w).max())


def test_watchdog_fires_on_stall(gpu, monkeypatch):
    monkeypatch.setenv("PE_FAULT_INJECT", "stall")
    monkeypatch.setenv("PE_WATCHDOG_S", "0.5")
    with pytest.raises(RuntimeError, match="watchdog"):
        solve(EllipseProblem(200, 300), backend="hip")


def test_one_rank_stall_fails_the_job(gpu):
    """PE_FAULT_INJECT=stall@rank:1 (SURVEY §5 hang@rank hook): rank 1's host
    loop never sees the device finish, its watchdog fires, the process exits
    non-zero and torchrun tears the job down — the job fails, it does not
    hang (the process group is killed if it ever did)."""
    import signal

    from conftest import free_port

    env = dict(os.environ, PE_COMM="host", PE_FAULT_INJECT="stall@rank:1", PE_WATCHDOG_S="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
           "poisson_ellipse_openmp_mpi_cuda_amd", "--quiet", "200", "300"]
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=90)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        pytest.fail("a stalled rank hung the job instead of failing it")
    assert p.returncode != 0
    assert "watchdog" in err, err[-3000:]


@pytest.mark.parametrize("algo", ["fused", "classic"])
def test_checkpoint_resume_bitwise(gpu, algo, tmp_path):
    prob = EllipseProblem(400, 600)
    ck = str(tmp_path / "ck")
    full = solve(prob, backend="hip", return_w=True, algo=algo, checkpoint=ck, checkpoint_every=200, chunk=8)
    assert full.iters == 546 and os.path.exists(ck + ".r0")
    res = solve(prob, backend="hip", return_w=True, algo=algo, resume=ck, chunk=8)
    assert res.converged and res.iters == full.iters
    assert np.array_equal(res.w, full.w)


def test_resume_rejects_mismatch(gpu, tmp_path):
    ck = str(tmp_path / "ck")
    solve(EllipseProblem(200, 300), backend="hip", checkpoint=ck, checkpoint_every=50, chunk=8)
    with pytest.raises(RuntimeError, match="does not match"):
        solve(EllipseProblem(210, 300), backend="hip", resume=ck)


@pytest.mark.parametrize("algo", ["fused", "classic"])
def test_device_history_matches_cpu(gpu, algo):
    prob = EllipseProblem(200, 300)
    c = solve(prob, backend="serial", keep_history=True)
    d = solve(prob, backend="hip", keep_history=True, algo=algo)
    assert len(d.history) == d.iters == c.iters
    np.testing.assert_allclose(d.history, c.history, rtol=1e-6)
    assert d.history[-1] < prob.tol <= d.history[-2]


# ---- LDS-resident single sweep (resident.hip) -------------------------------
@pytest.mark.parametrize("M,N", [(40, 40), (257, 129), (400, 600), (800, 1200), (130, 1000), (1000, 130)])
def test_resident_matches_streaming(gpu, M, N, monkeypatch):
    """The resident kernel (tiles of 124 columns × R rows, one workgroup each,
    ring-2 exchange + 7 partial sums per iteration behind a grid barrier)
    against the streaming single sweep: same iteration count, same solution
    (different summation order only), golden counts on the published grids."""
    prob = EllipseProblem(M, N)
    monkeypatch.setenv("PE_RESIDENT", "0")
    ref = solve(prob, backend="hip", return_w=True, algo="fused")
    monkeypatch.delenv("PE_RESIDENT")
    res = solve(prob, backend="hip", return_w=True)
    assert res.algo == "resident" and ref.algo == "fused"
    assert res.iters == ref.iters
    if (M, N, "weighted") in GOLDEN_ITERS:
        assert res.iters == GOLDEN_ITERS[(M, N, "weighted")]
    np.testing.assert_allclose(res.w, ref.w, rtol=0, atol=1e-10)
    assert res.l2_err == pytest.approx(ref.l2_err, rel=1e-7)


def test_resident_barrier_timeout_falls_back(gpu, monkeypatch):
    """A resident launch whose grid barrier times out (PE_FAULT_INJECT=resbarrier:
    one workgroup never arrives; 0.1 s limit) aborts with nothing written
    back; the solver clears the abort, switches to the streaming sweep and
    still converges in the golden count (reference iteration must complete:
    poisson_mpi_decomp.cpp:400-457)."""
    monkeypatch.setenv("PE_FAULT_INJECT", "resbarrier")
    monkeypatch.setenv("PE_RES_TIMEOUT_S", "0.1")
    rep = solve(EllipseProblem(800, 1200), backend="hip")
    assert rep.resident_fallback and rep.algo == "fused (resident fallback)"
    assert rep.converged and rep.iters == 989
    assert rep.l2_err == pytest.approx(1.92e-4, rel=5e-3)


def test_resident_late_workgroup_restarts(gpu, monkeypatch):
    """A workgroup that arrives at the grid barrier AFTER the others timed out
    (PE_FAULT_INJECT=reslate) passes it and writes its tile back while the
    rest aborted: the launch's state is not resumable.  The sticky res_abort
    makes the solver start over on the streaming sweep, and w equals a
    streaming solve's (resident.hip:454)."""
    prob = EllipseProblem(800, 1200)
    monkeypatch.setenv("PE_RESIDENT", "0")
    ref = solve(prob, backend="hip", return_w=True, algo="fused")
    monkeypatch.delenv("PE_RESIDENT")
    monkeypatch.setenv("PE_FAULT_INJECT", "reslate")
    monkeypatch.setenv("PE_RES_TIMEOUT_S", "0.1")
    rep = solve(prob, backend="hip", return_w=True)
    assert rep.resident_fallback and rep.algo == "fused (resident fallback)"
    assert rep.converged and rep.iters == ref.iters == 989
    np.testing.assert_allclose(rep.w, ref.w, rtol=0, atol=1e-12)


@pytest.mark.parametrize("M,N,chunk,max_iter", [(800, 1200, 988, 0), (300, 700, 512, 513)])
def test_resident_terminal_at_launch_start(gpu, M, N, chunk, max_iter, monkeypatch):
    """The solve ends on the FIRST iteration of a resident launch (convergence at
    989 with 988-iteration launches; the cap 513 with 512): workgroup 0 writes
    the terminal state only after every workgroup has read the entry state,
    so every tile adds its α·p and the result equals the streaming sweep's."""
    prob = EllipseProblem(M, N)
    if max_iter:
        prob.max_iter = max_iter
    monkeypatch.setenv("PE_RESIDENT", "0")
    ref = solve(prob, backend="hip", return_w=True, chunk=chunk, algo="fused")
    monkeypatch.delenv("PE_RESIDENT")
    res = solve(prob, backend="hip", return_w=True, chunk=chunk)
    assert res.algo == "resident" and ref.algo == "fused"
    assert res.iters == ref.iters == (max_iter or 989)
    np.testing.assert_allclose(res.w, ref.w, rtol=0, atol=1e-10)


@pytest.mark.parametrize("parts", [[60], [7, 13, 40], [1, 1, 58]])
def test_resident_launch_split_bitwise(gpu, nat, parts):
    """A resident launch starts from and ends in the streaming layout/state:
    how the iterations are split into launches does not change one bit."""
    prob = EllipseProblem(300, 700)
    blk = D.block(300, 700, 1, 0)
    out = []
    for split in ([60], parts):
        opt = nat.SolveOptions()
        opt.check_tol = False
        opt.chunk = 1 << 20
        s = nat.DeviceSolver(prob.to_native(), blk, None, opt)
        assert s.resident
        s.reset()
        for n in split:
            s.run_iterations(n, True)
        s.synchronize()
        out.append((s.state(), s.w()))
    (a, wa), (b, wb) = out
    assert a["iter"] == b["iter"] == 60
    # the live sums are those of the last iteration (parity 1 after 60 from parity 0)
    assert a["fs"][1] == b["fs"][1] and a["alpha"] == b["alpha"] and a["gprev"] == b["gprev"]
    assert np.array_equal(wa, wb)


def test_resident_state_matches_streaming_kernel(gpu, nat, monkeypatch):
    """α, β and the 7 sums after 25 resident iterations agree with the
    streaming kernel's to rounding (the recurrence is the same)."""
    prob = EllipseProblem(400, 600)
    blk = D.block(400, 600, 1, 0)
    st = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PE_RESIDENT", flag)
        opt = nat.SolveOptions()
        opt.check_tol = False
        opt.algo = 2 if flag == "0" else 0
        s = nat.DeviceSolver(prob.to_native(), blk, None, opt)
        assert s.resident == (flag == "1")
        s.reset()
        s.run_iterations(25, False)
        s.synchronize()
        st[flag] = (s.state(), s.w())
    (a, wa), (b, wb) = st["1"], st["0"]
    assert a["iter"] == b["iter"] == 25
    assert a["alpha"] == pytest.approx(b["alpha"], rel=1e-11)
    assert a["beta"] == pytest.approx(b["beta"], rel=1e-11)
    np.testing.assert_allclose(wa, wb, rtol=0, atol=1e-13 * np.abs(wb).max())


# ---- production single-sweep kernels vs the PyTorch fp64 recurrence ---------
@pytest.mark.parametrize("M,N", [(300, 420), (257, 129)])
@pytest.mark.parametrize("kernel", ["streaming", "resident"])
def test_production_sweep_vs_torch_recurrence(gpu, nat, M, N, kernel, monkeypatch):
    """S_0 + 20 sweeps of the production kernel (streaming kS, or the resident
    kernel), convergence test off: the 7 reduced sums, α, β and the r / p
    planes and w against torch_ref.single_sweep (reference operator,
    divisions; the kernels use the division-free coefficient path) —
    reference iteration: stage2-mpi/poisson_mpi_decomp.cpp:400-457."""
    K = 20
    monkeypatch.setenv("PE_RESIDENT", "1" if kernel == "resident" else "0")
    prob = EllipseProblem(M, N)
    opt = nat.SolveOptions()
    opt.algo = 2
    opt.check_tol = False
    s = nat.DeviceSolver(prob.to_native(), D.block(M, N, 1, 0), None, opt)
    assert s.resident == (kernel == "resident")
    s.reset()
    s.run_iterations(K, False)
    s.synchronize()
    st = s.state()
    ref = torch_ref.single_sweep(prob, K)
    par = (K - 1) & 1
    got, want = st["fs"][par], ref.sums[K]
    scale = max(abs(x) for x in want)
    for n in range(7):
        assert got[n] == pytest.approx(want[n], rel=1e-10, abs=1e-13 * scale), n
    assert st["alpha"] == pytest.approx(ref.alpha[-1], rel=1e-12)
    assert st["beta"] == pytest.approx(ref.beta[-1], rel=1e-12)
    fields = {"r": s.field(0 if par == 0 else 4), "p": s.field(2 if par == 0 else 3)}
    for name, f in fields.items():
        want_f = getattr(ref, name)[1:M, 1:N].numpy()
        np.testing.assert_allclose(f[2:M + 1, 2:N + 1], want_f, rtol=0, atol=1e-12 * np.abs(want_f).max(),
                                   err_msg=name)
    wref = ref.w[1:M, 1:N].numpy()
    np.testing.assert_allclose(s.w(), wref, rtol=0, atol=1e-12 * np.abs(wref).max())


def test_virtual_split_sweep_vs_torch_recurrence(gpu):
    """2x2 virtual ranks (halo exchange, strips that cut boundary-band rows)
    through the streaming kernel: w after 20 sweeps against the recurrence."""
    prob = EllipseProblem(300, 420)
    prob.max_iter = 20
    rep = solve(prob, backend="hip-group", ranks=4, decomp="2x2", return_w=True, check_tol=False, algo="fused")
    assert rep.iters == 20 and rep.Px * rep.Py == 4
    wref = torch_ref.single_sweep(EllipseProblem(300, 420), 20).w[1:300, 1:420].numpy()
    np.testing.assert_allclose(rep.w, wref, rtol=0, atol=1e-12 * np.abs(wref).max())


@pytest.mark.parametrize("M,N,kw", [(40, 40, {}), (257, 129, {}), (800, 1200, {}),
                                    (300, 200, dict(A1=-2.0, B1=2.0, A2=-1.0, B2=1.0, cx=0.25, cy=1.0))])
def test_fast_coefficients_vs_assembly(gpu, nat, M, N, kw):
    """The single-sweep kernels' division-free coefficients (cset_rc: t = l·(1/h),
    t + (1-t)·(1/eps), reciprocal + Newton 1/D) against the reference assembly
    (fic_reg_local, poisson_mpi_decomp.cpp:124-170).  Interior / exterior faces
    are exact; a cut face's blend amplifies the one-rounding difference of t
    by 1/eps, so it is held to (1/eps)·ulp(1) + 2 ulp; 1/D (a sum of faces ≥ 1
    each, then a reciprocal) to a relative (1/eps)·ulp(1) + 4 ulp."""
    prob = EllipseProblem(M, N, **kw)
    a, b, di = (np.asarray(x) for x in nat.device_coefficients_fast(prob.to_native(), D.block(M, N, 1, 0)))
    at, bt, _ = torch_ref.assemble(prob)
    Dt = torch_ref.diag(at, bt, prob.h1, prob.h2).numpy()
    at, bt = at.numpy(), bt.numpy()
    assert a.shape == at.shape == (M + 1, N + 1)
    inv_eps = 1.0 / prob.eps
    plain_a = (at == 1.0) | (at == inv_eps)
    plain_b = (bt == 1.0) | (bt == inv_eps)
    assert np.array_equal(a[plain_a], at[plain_a]) and np.array_equal(b[plain_b], bt[plain_b])
    bound = lambda ref: inv_eps * np.spacing(1.0) + 2 * np.spacing(np.abs(ref))  # noqa: E731
    assert np.all(np.abs(a - at) <= bound(at))
    assert np.all(np.abs(b - bt) <= bound(bt))
    assert plain_a.sum() < a.size  # band faces exist
    dref = 1.0 / Dt[1:M, 1:N]
    rel = np.abs(di[1:M, 1:N] - dref) / dref
    assert rel.max() <= (inv_eps + 4.0) * np.spacing(1.0)


@pytest.mark.parametrize("spec,P", [("4x2", 8), ("2x2", 4), ("8x1", 8), ("4x1", 4)])
def test_overlap_async_loopback_transport_bitwise(gpu, monkeypatch, spec, P):
    """the halo/interior overlap through an
    ASYNCHRONOUS transport that moves data, on 2-D blocks AND on the row slabs
    that the multi-GPU default runs (kSignal on slabs: one phase).  The
    loopback delay transport waits 150 µs on the stream (longer than a sweep
    of this block), then copies every send buffer into its receive buffer with
    a stream-ordered device copy — no host synchronisation anywhere, as with
    RCCL.  The peer-put kernel in loopback (PE_PUT_LOOPBACK=1: the rank is its
    own peer, each message lands in its own receive buffer through the inbox,
    flags and all) moves the same data.  Every arm — exchange or put,
    serialised on the solver stream (PE_OV_DEBUG=2), overlapped (kWaitSig →
    pack → exchange → unpack on the halo stream → event → next sweep), or with
    no overlap at all — must end bitwise where the serialised exchange does:
    any ordering hole (the pack before the boundary items' stores, the next
    sweep before the unpack, a put read before its flag) changes the data."""
    from poisson_ellipse_openmp_mpi_cuda_amd._loader import native
    from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

    nat = native()
    M = N = 1024
    prob = EllipseProblem(M, N)
    g = D.grid(P, M, N, spec)
    blk = nat.decompose(M, N, g, P // 2)
    out = {}
    for halo in ("exchange", "put"):
        for ov, dbg in (("1", "2"), ("1", "0"), ("0", "0")):
            monkeypatch.setenv("PE_HALO", halo)
            monkeypatch.setenv("PE_PUT_LOOPBACK", "1" if halo == "put" else "0")
            monkeypatch.setenv("PE_OVERLAP", ov)
            monkeypatch.setenv("PE_OV_DEBUG", dbg)
            opt = nat.SolveOptions()
            opt.check_tol = False
            comm = nat.make_delay_comm(P, 150.0, 3.0, True)
            s = nat.DeviceSolver(prob.to_native(), blk, comm, opt)
            assert s.overlap == (ov == "1") and s.sweep_steps == 3
            assert s.halo_put == (halo == "put"), (s.halo_path, s.put_status)
            assert s.halo_path.startswith(halo + ("+overlap" if ov == "1" else "")), s.halo_path
            s.reset()
            s.run_iterations(45, False)
            s.synchronize()
            out[(halo, ov, dbg)] = (s.state(), s.w())
            del s, comm
    # (the overlap lays out its boundary items first — other per-block partial
    # sums, other rounding — so each arm is compared within its layout: the
    # overlapped arms against the serialised exchange of the same layout, the
    # put without overlap against the exchange without overlap)
    for ref, keys in ((("exchange", "1", "2"), [("exchange", "1", "0"), ("put", "1", "2"), ("put", "1", "0")]),
                      (("exchange", "0", "0"), [("put", "0", "0")])):
        st0, w0 = out[ref]
        for key in keys:
            st1, w1 = out[key]
            assert st0["iter"] == st1["iter"] and st0["status"] == st1["status"], key
            assert st0["fs2"] == st1["fs2"], key
            np.testing.assert_array_equal(w0, w1, err_msg=str(key))
    # across the layouts: the same iterate to rounding
    wa, wb = out[("exchange", "1", "2")][1], out[("exchange", "0", "0")][1]
    np.testing.assert_allclose(wa, wb, rtol=0, atol=1e-11 * np.abs(wb).max())


def test_halo_path_choice_follows_the_transport(gpu, monkeypatch):
    """the multi-rank halo path is chosen at construction by
    timing the candidates on the job's transport (here one rank's block of an
    8-rank row-slab split of 4096², the loopback forms of the put and the push
    on one GPU, the delay transport as the exchange).  The pick is the fastest
    candidate as timed; with a 3 ms exchange every exchange arm loses to the
    put / push; PE_HALO=exchange with a 400 µs exchange picks the faster of
    the two exchange arms (on this small block, one item per wave, the boundary
    items end with the sweep and the overlap hides next to nothing: 474 vs 463
    µs per sweep, round 6); the overlap arms are timed at the rows-per-item
    tuning's best heights ("exchange+overlap @96"); PE_HALO_TUNE=0 times
    nothing."""
    from poisson_ellipse_openmp_mpi_cuda_amd._loader import native
    from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

    nat = native()
    M = N = 4096
    prob = EllipseProblem(M, N)
    blk = nat.decompose(M, N, D.grid(8, M, N, "8x1"), 3)
    monkeypatch.delenv("PE_OVERLAP", raising=False)
    monkeypatch.delenv("PE_HALO", raising=False)
    monkeypatch.setenv("PE_PUT_LOOPBACK", "1")
    monkeypatch.setenv("PE_PUSH_LOOPBACK", "1")

    def build(ex_us):
        opt = nat.SolveOptions()
        comm = nat.make_delay_comm(8, ex_us, 0.0, True)
        return nat.DeviceSolver(prob.to_native(), blk, comm, opt), comm

    def final_times(cands):  # a finalist's time is the min of its two timings
        final = {}  # (an overlap arm timed at two heights: "exchange+overlap @96")
        for n, us in cands:
            base = n.replace(" (again)", "").split(" @")[0]
            final[base] = min(final.get(base, us), us)
        return final

    s, c = build(0.0)
    cands = s.halo_candidates
    names = [n.split(" @")[0] for n, _ in cands]
    for want in ("exchange", "exchange+overlap", "put", "put+overlap", "push"):
        assert want in names, names
    final = final_times(cands)
    assert s.halo_path == min(final, key=final.get), (s.halo_path, cands)
    del s, c
    s, c = build(3000.0)
    assert s.halo_path in ("put", "put+overlap", "push"), (s.halo_path, s.halo_candidates)
    ex = [us for n, us in s.halo_candidates if n.startswith("exchange")]
    assert min(ex) > 3000.0
    del s, c
    monkeypatch.setenv("PE_HALO", "exchange")
    s, c = build(400.0)
    assert {n.replace(" (again)", "").split(" @")[0] for n, _ in s.halo_candidates} == {"exchange", "exchange+overlap"}
    assert s.halo_path == min(final_times(s.halo_candidates), key=final_times(s.halo_candidates).get)
    assert s.overlap == (s.halo_path == "exchange+overlap")
    del s, c
    monkeypatch.setenv("PE_HALO_TUNE", "0")
    s, c = build(400.0)
    assert s.halo_candidates == [] and s.halo_path == "exchange (PE_HALO_TUNE=0)" and not s.overlap


def test_diagnostic_knobs(gpu, monkeypatch):
    """The diagnostic / set-up knobs the knob table keeps (docs/PERFORMANCE.md),
    each exercised once: PE_STAMPS=1 (three-step stamps) and PE_RES_STAMPS=1
    (resident kernel) record s_memrealtime stamps; PE_TI_TUNE=0 skips the
    rows-per-item tuning; PE_PLACEMENT_TRIES=1 skips the placement search;
    PE_TIMER_SAMPLE=0 turns the sampled phase timers off (T_gpu is then the
    loop's device span); PE_CTOR_TRACE=1 prints the construction phases."""
    from poisson_ellipse_openmp_mpi_cuda_amd._loader import native
    from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

    nat = native()

    def make(M, N, **env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        opt = nat.SolveOptions()
        opt.check_tol = False
        s = nat.DeviceSolver(EllipseProblem(M, N).to_native(), D.block(M, N, 1, 0), None, opt)
        for k in env:
            monkeypatch.delenv(k)
        return s

    s = make(1024, 1024, PE_STAMPS="1", PE_RESIDENT="0")
    assert s.sweep_steps == 3
    s.reset()
    s.run_iterations(9, False)
    st = np.asarray(s.stamps(), dtype=np.uint64)
    assert st.size > 0 and np.count_nonzero(st) > 0
    s = make(400, 600, PE_RES_STAMPS="1")
    assert s.resident
    s.reset()
    s.run_iterations(16, False)
    st = np.asarray(s.stamps(), dtype=np.uint64)
    assert st.size > 0 and np.count_nonzero(st) > 0
    tuned = make(1600, 2400)
    assert len(tuned.ti_tuning_ms) > 0
    untuned = make(1600, 2400, PE_TI_TUNE="0")
    assert len(untuned.ti_tuning_ms) == 0
    one = make(8192, 8192, PE_PLACEMENT_TRIES="1")
    assert len(one.placement_ms) == 0
    del one
    monkeypatch.setenv("PE_TIMER_SAMPLE", "0")
    rep = solve(EllipseProblem(400, 600), backend="hip", algo="three-step")
    assert rep.iters == 546 and rep.timers["sampled"] == 0 and rep.timers["gpu"] > 0
    monkeypatch.delenv("PE_TIMER_SAMPLE")
    env = dict(os.environ, PE_CTOR_TRACE="1")
    out = subprocess.run([os.path.join(ROOT, "bin", "pe_hip"), "--json", "400", "600"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "[pe] ctor" in out.stderr and "halo path" in out.stderr

"""MI355X tests of the three-step sweep (csrc/hip/fused3.hip): three PCG
iterations per pass over memory, one 19-sum reduction per three iterations,
late stop tests with a w fix-up launch.

Checked against the reference iteration counts (stage2-mpi/
poisson_mpi_decomp.cpp:400-457 via the survey's golden values), the PyTorch
fp64 recurrence (torch_ref.three_step, itself equal to the single-sweep
recurrence to rounding) and the single-sweep kernel in every terminal case:
convergence on the first / second / third iteration of a sweep (1858, 989 and
546 iterations: 1858 ≡ 1, 989 ≡ 2, 546 ≡ 0 mod 3), the iteration cap,
breakdown and non-finite scalars."""

import os

import numpy as np
import pytest

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve
from poisson_ellipse_openmp_mpi_cuda_amd.models.ellipse import GOLDEN_ITERS, GOLDEN_L2
from poisson_ellipse_openmp_mpi_cuda_amd.ops import torch_ref
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

pytestmark = pytest.mark.gpu
THREE = "three-step"


@pytest.mark.parametrize("M,N,norm", [(40, 40, "weighted"), (40, 40, "unweighted"), (400, 600, "weighted"),
                                      (800, 1200, "weighted"), (1600, 2400, "weighted"), (2048, 2048, "weighted"),
                                      (2400, 3200, "weighted"), (10, 10, "unweighted"), (20, 20, "unweighted")])
def test_three_step_golden_iterations(gpu, M, N, norm):
    rep = solve(EllipseProblem(M, N, norm=norm), backend="hip", algo=THREE)
    assert rep.algo == "three-step"
    assert rep.converged and rep.iters == GOLDEN_ITERS[(M, N, norm)]
    if (M, N) in GOLDEN_L2 and norm == "weighted":
        assert rep.l2_err == pytest.approx(GOLDEN_L2[(M, N)], rel=5e-3)


@pytest.mark.parametrize("M,N", [(4096, 4096), (8192, 8192)])
def test_three_step_large_golden(gpu, M, N):
    rep = solve(EllipseProblem(M, N), backend="hip", algo=THREE)
    assert rep.converged and rep.iters == GOLDEN_ITERS[(M, N, "weighted")]
    assert rep.l2_err == pytest.approx(GOLDEN_L2[(M, N)], rel=5e-3)


def _solver(nat, prob, **kw):
    opt = nat.SolveOptions()
    opt.algo = 4
    opt.check_tol = False
    for k, v in kw.items():
        setattr(opt, k, v)
    M, N = prob.M, prob.N
    return nat.DeviceSolver(prob.to_native(), D.block(M, N, 1, 0), None, opt)


@pytest.mark.parametrize("M,N", [(300, 420), (257, 129), (130, 1000)])
def test_three_step_sweeps_vs_torch_recurrence(gpu, nat, M, N):
    """S_0 + 8 sweeps (24 iterations) of kS3, convergence test off: the 19
    reduced sums, α₃, β₃, the r / p planes and w against torch_ref.three_step
    (reference operator, divisions; the kernel uses the division-free
    coefficients)."""
    J = 8
    prob = EllipseProblem(M, N)
    s = _solver(nat, prob)
    assert s.sweep_steps == 3
    s.reset()
    s.run_iterations(3 * J, False)
    s.synchronize()
    st = s.state()
    assert st["iter"] == 3 * J and st["status"] == 0
    ref = torch_ref.three_step(prob, J)
    par = (J - 1) & 1
    got, want = st["fs2"][par], ref.sums[J]
    scale = max(abs(x) for x in want)
    for n in range(19):
        assert got[n] == pytest.approx(want[n], rel=1e-9, abs=1e-12 * scale), n
    assert st["alpha"] == pytest.approx(ref.alpha[-1][2], rel=1e-11)
    assert st["beta"] == pytest.approx(ref.beta[-1][2], rel=1e-11)
    fields = {"r": s.field(0 if par == 0 else 4), "p": s.field(2 if par == 0 else 3)}
    for name, f in fields.items():
        want_f = getattr(ref, name)[1:M, 1:N].numpy()
        np.testing.assert_allclose(f[2:M + 1, 2:N + 1], want_f, rtol=0, atol=1e-11 * np.abs(want_f).max(),
                                   err_msg=name)
    wref = ref.w[1:M, 1:N].numpy()
    np.testing.assert_allclose(s.w(), wref, rtol=0, atol=1e-11 * np.abs(wref).max())


@pytest.mark.parametrize("n", [1, 2, 4, 20, 23])
def test_three_step_partial_sweeps(gpu, nat, n):
    """run_iterations(n) with 3 ∤ n ends with a partial sweep (KParams::mlimit):
    exactly n iterations, and w equals the single sweep's after n iterations."""
    prob = EllipseProblem(300, 420)
    s = _solver(nat, prob)
    s.reset()
    s.run_iterations(n, False)
    s.synchronize()
    st = s.state()
    assert st["iter"] == n and st["status"] == 0
    ref = torch_ref.single_sweep(prob, n)
    wref = ref.w[1:300, 1:420].numpy()
    np.testing.assert_allclose(s.w(), wref, rtol=0, atol=1e-11 * np.abs(wref).max())
    # and the run continues from there: n + 6 iterations in two calls = in one
    s.run_iterations(6, False)
    s.synchronize()
    assert s.state()["iter"] == n + 6


@pytest.mark.parametrize("M,N", [(40, 40), (400, 600), (800, 1200), (1600, 2400), (257, 129)])
def test_three_step_matches_single_sweep(gpu, M, N, monkeypatch):
    """Same iteration count and solution as the single sweep; 800×1200 (989)
    and 1600×2400 (1858) stop on the second / first iteration of a sweep: the
    fix-up launch takes the later iterations back out of w."""
    monkeypatch.setenv("PE_RESIDENT", "0")
    prob = EllipseProblem(M, N)
    a = solve(prob, backend="hip", return_w=True, algo="fused")
    b = solve(prob, backend="hip", return_w=True, algo=THREE)
    assert a.iters == b.iters
    np.testing.assert_allclose(b.w, a.w, rtol=0, atol=1e-10)
    assert b.l2_err == pytest.approx(a.l2_err, rel=1e-7)


@pytest.mark.parametrize("cap", [7, 8, 9, 1, 2, 3])
def test_three_step_iteration_cap(gpu, cap, monkeypatch):
    """A cap that is not a multiple of 3 ends on a partial sweep; w equals the
    single sweep's."""
    monkeypatch.setenv("PE_RESIDENT", "0")
    prob = EllipseProblem(300, 420)
    prob.max_iter = cap
    a = solve(prob, backend="hip", return_w=True, algo="fused")
    b = solve(prob, backend="hip", return_w=True, algo=THREE)
    assert a.iters == b.iters == cap and not b.converged
    np.testing.assert_allclose(b.w, a.w, rtol=0, atol=1e-12 * np.abs(a.w).max())


def test_three_step_history_matches_cpu(gpu):
    prob = EllipseProblem(200, 300)
    c = solve(prob, backend="serial", keep_history=True)
    d = solve(prob, backend="hip", keep_history=True, algo=THREE)
    assert len(d.history) == d.iters == c.iters
    np.testing.assert_allclose(d.history, c.history, rtol=1e-6)


def test_three_step_bitwise_deterministic_and_graph_equivalent(gpu):
    prob = EllipseProblem(500, 700)
    a = solve(prob, backend="hip", return_w=True, algo=THREE)
    b = solve(prob, backend="hip", return_w=True, algo=THREE)
    c = solve(prob, backend="hip", return_w=True, algo=THREE, graph=True)
    assert a.iters == b.iters == c.iters
    assert np.array_equal(a.w, b.w) and np.array_equal(a.w, c.w)


def test_three_step_checkpoint_resume_bitwise(gpu, tmp_path):
    prob = EllipseProblem(400, 600)
    ck = str(tmp_path / "ck")
    full = solve(prob, backend="hip", return_w=True, algo=THREE, checkpoint=ck, checkpoint_every=200, chunk=12)
    assert full.iters == 546 and os.path.exists(ck + ".r0")
    res = solve(prob, backend="hip", return_w=True, algo=THREE, resume=ck, chunk=12)
    assert res.converged and res.iters == full.iters
    assert np.array_equal(res.w, full.w)
    with pytest.raises(RuntimeError, match="has the three-step layout.*pass --algo three-step"):  # not resumable here
        solve(prob, backend="hip", algo="two-step", resume=ck)
    # a layout code this build does not know (header field `fused`, byte 32):
    # a readable error, never an out-of-range table lookup
    raw = bytearray(open(ck + ".r0", "rb").read())
    raw[32:36] = (9).to_bytes(4, "little", signed=True)
    bad = str(tmp_path / "bad")
    open(bad + ".r0", "wb").write(bytes(raw))
    with pytest.raises(RuntimeError, match=r"has the unknown \(steps=9\) layout.*runs three-step"):
        solve(prob, backend="hip", algo=THREE, resume=bad)


def test_three_step_breakdown_and_nonfinite(gpu, monkeypatch):
    """zero@iter:20 zeroes the (p, Ap) moments of the sweep completing
    iterations 19..21: iteration 22 (the next sweep's first) breaks down before
    its update and w is the 21-iteration one; nan@iter stops with a non-finite
    status."""
    prob = EllipseProblem(200, 300)
    monkeypatch.setenv("PE_FAULT_INJECT", "zero@iter:20")
    brk = solve(prob, backend="hip", return_w=True, algo=THREE)
    assert brk.breakdown and not brk.converged and brk.iters == 22
    monkeypatch.setenv("PE_FAULT_INJECT", "nan@iter:20")
    bad = solve(prob, backend="hip", algo=THREE)
    assert bad.nonfinite and 22 <= bad.iters <= 24
    monkeypatch.delenv("PE_FAULT_INJECT")
    capped = EllipseProblem(200, 300)
    capped.max_iter = 21
    ref = solve(capped, backend="hip", return_w=True, algo=THREE)
    np.testing.assert_array_equal(brk.w, ref.w)


def test_three_step_random_init(gpu):
    prob = EllipseProblem(200, 300)
    c = solve(prob, backend="serial", init="random", seed=11, return_w=True)
    d = solve(prob, backend="hip", init="random", seed=11, return_w=True, algo=THREE)
    assert abs(c.iters - d.iters) <= 1
    np.testing.assert_allclose(d.w, c.w, rtol=0, atol=1e-9)


def test_three_step_is_auto_default(gpu, monkeypatch):
    """auto picks the three-step sweep for a single-rank block the resident
    kernel cannot hold; PE_STEPS=2 keeps the two-step sweep."""
    prob = EllipseProblem(1600, 2400)
    assert solve(prob, backend="hip").algo == "three-step"
    monkeypatch.setenv("PE_STEPS", "2")
    assert solve(prob, backend="hip").algo == "two-step"


@pytest.mark.parametrize("ranks,decomp", [(2, "1x2"), (4, "2x2"), (6, "2x3"), (3, "rows")])
def test_three_step_virtual_ranks(gpu, ranks, decomp):
    """Virtual ranks on one GPU (backend hip-group) run the three-step sweep
    on blocks of >= 12 x 12: the group driver packs and exchanges the 6-deep
    halos after every sweep and sums the 19 sums over the blocks; the last
    strip of a block with an UP neighbour keeps that neighbour's columns out
    of its sums.  Same iteration count and w as one block."""
    prob = EllipseProblem(300, 437)
    one = solve(prob, backend="hip", return_w=True, algo=THREE)
    grp = solve(prob, backend="hip-group", ranks=ranks, decomp=decomp, return_w=True)
    assert grp.algo == "three-step" and grp.Px * grp.Py == ranks
    assert abs(grp.iters - one.iters) <= 1 and grp.converged
    np.testing.assert_allclose(grp.w, one.w, rtol=0, atol=1e-9)


@pytest.mark.parametrize("cap", [7, 8, 9])
def test_three_step_virtual_ranks_cap(gpu, cap):
    """An iteration cap inside a sweep: the group stops on it like one block."""
    prob = EllipseProblem(300, 437)
    prob.max_iter = cap
    one = solve(prob, backend="hip", return_w=True, algo=THREE)
    grp = solve(prob, backend="hip-group", ranks=4, decomp="2x2", return_w=True)
    assert grp.algo == "three-step" and grp.iters == one.iters == cap and not grp.converged
    np.testing.assert_allclose(grp.w, one.w, rtol=0, atol=1e-12 * np.abs(one.w).max())


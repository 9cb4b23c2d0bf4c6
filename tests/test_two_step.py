"""MI355X tests of the two-step sweep (csrc/hip/fused2.hip): two PCG
iterations per pass over memory, one 20-sum reduction per two iterations.

Checked against the reference iteration counts (stage2-mpi/
poisson_mpi_decomp.cpp:400-457 via the survey's golden values), the PyTorch
fp64 recurrence (torch_ref.two_step, itself equal to the single-sweep
recurrence to rounding) and the single-sweep kernel (every terminal case:
convergence / cap / breakdown on the first or the second iteration of a
sweep)."""

import os

import numpy as np
import pytest

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve
from poisson_ellipse_openmp_mpi_cuda_amd.models.ellipse import GOLDEN_ITERS, GOLDEN_L2
from poisson_ellipse_openmp_mpi_cuda_amd.ops import torch_ref
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

pytestmark = pytest.mark.gpu
TWO = "two-step"


@pytest.mark.parametrize("M,N,norm", [(40, 40, "weighted"), (40, 40, "unweighted"), (400, 600, "weighted"),
                                      (800, 1200, "weighted"), (1600, 2400, "weighted"), (2048, 2048, "weighted"),
                                      (10, 10, "unweighted"), (20, 20, "unweighted")])
def test_two_step_golden_iterations(gpu, M, N, norm):
    rep = solve(EllipseProblem(M, N, norm=norm), backend="hip", algo=TWO)
    assert rep.algo == "two-step"
    assert rep.converged and rep.iters == GOLDEN_ITERS[(M, N, norm)]
    if (M, N) in GOLDEN_L2 and norm == "weighted":
        assert rep.l2_err == pytest.approx(GOLDEN_L2[(M, N)], rel=5e-3)


@pytest.mark.parametrize("M,N", [(4096, 4096), (8192, 8192)])
def test_two_step_large_golden(gpu, M, N):
    rep = solve(EllipseProblem(M, N), backend="hip", algo=TWO)
    assert rep.converged and rep.iters == GOLDEN_ITERS[(M, N, "weighted")]
    assert rep.l2_err == pytest.approx(GOLDEN_L2[(M, N)], rel=5e-3)


@pytest.mark.parametrize("M,N", [(300, 420), (257, 129), (130, 1000)])
def test_two_step_sweeps_vs_torch_recurrence(gpu, nat, M, N):
    """S_0 + 10 sweeps (20 iterations) of kS2, convergence test off: the 20
    reduced sums, α₂, β₂, the r / p planes and w against torch_ref.two_step
    (reference operator, divisions; the kernel uses the division-free
    coefficients)."""
    J = 10
    prob = EllipseProblem(M, N)
    opt = nat.SolveOptions()
    opt.algo = 3
    opt.check_tol = False
    s = nat.DeviceSolver(prob.to_native(), D.block(M, N, 1, 0), None, opt)
    assert s.two_step
    s.reset()
    s.run_iterations(2 * J, False)
    s.synchronize()
    st = s.state()
    assert st["iter"] == 2 * J and st["status"] == 0
    ref = torch_ref.two_step(prob, J)
    par = (J - 1) & 1
    got, want = st["fs2"][par], ref.sums[J]
    scale = max(abs(x) for x in want)
    for n in range(20):
        assert got[n] == pytest.approx(want[n], rel=1e-9, abs=1e-12 * scale), n
    assert st["alpha"] == pytest.approx(ref.alpha[-1][1], rel=1e-11)
    assert st["beta"] == pytest.approx(ref.beta[-1][1], rel=1e-11)
    fields = {"r": s.field(0 if par == 0 else 4), "p": s.field(2 if par == 0 else 3)}
    for name, f in fields.items():
        want_f = getattr(ref, name)[1:M, 1:N].numpy()
        np.testing.assert_allclose(f[2:M + 1, 2:N + 1], want_f, rtol=0, atol=1e-11 * np.abs(want_f).max(),
                                   err_msg=name)
    wref = ref.w[1:M, 1:N].numpy()
    np.testing.assert_allclose(s.w(), wref, rtol=0, atol=1e-11 * np.abs(wref).max())


@pytest.mark.parametrize("M,N", [(40, 40), (400, 600), (800, 1200), (257, 129)])
def test_two_step_matches_single_sweep(gpu, M, N, monkeypatch):
    """Same iteration count and solution as the single sweep; 800×1200 stops
    on the FIRST iteration of a sweep (989 is odd: w += α₁p₁ only)."""
    monkeypatch.setenv("PE_RESIDENT", "0")
    prob = EllipseProblem(M, N)
    a = solve(prob, backend="hip", return_w=True, algo="fused")
    b = solve(prob, backend="hip", return_w=True, algo=TWO)
    assert a.iters == b.iters
    np.testing.assert_allclose(b.w, a.w, rtol=0, atol=1e-10)
    assert b.l2_err == pytest.approx(a.l2_err, rel=1e-7)


@pytest.mark.parametrize("cap", [7, 8, 1, 2])
def test_two_step_iteration_cap(gpu, cap, monkeypatch):
    """An odd cap ends on a sweep's first iteration (pointwise w += α₁p₁), an
    even one after the full sweep; w equals the single sweep's."""
    monkeypatch.setenv("PE_RESIDENT", "0")
    prob = EllipseProblem(300, 420)
    prob.max_iter = cap
    a = solve(prob, backend="hip", return_w=True, algo="fused")
    b = solve(prob, backend="hip", return_w=True, algo=TWO)
    assert a.iters == b.iters == cap and not b.converged
    np.testing.assert_allclose(b.w, a.w, rtol=0, atol=1e-12 * np.abs(a.w).max())


def test_two_step_history_matches_cpu(gpu):
    prob = EllipseProblem(200, 300)
    c = solve(prob, backend="serial", keep_history=True)
    d = solve(prob, backend="hip", keep_history=True, algo=TWO)
    assert len(d.history) == d.iters == c.iters
    np.testing.assert_allclose(d.history, c.history, rtol=1e-6)


def test_two_step_bitwise_deterministic_and_graph_equivalent(gpu):
    prob = EllipseProblem(500, 700)
    a = solve(prob, backend="hip", return_w=True, algo=TWO)
    b = solve(prob, backend="hip", return_w=True, algo=TWO)
    c = solve(prob, backend="hip", return_w=True, algo=TWO, graph=True)
    assert a.iters == b.iters == c.iters
    assert np.array_equal(a.w, b.w) and np.array_equal(a.w, c.w)


def test_two_step_checkpoint_resume_bitwise(gpu, tmp_path):
    prob = EllipseProblem(400, 600)
    ck = str(tmp_path / "ck")
    full = solve(prob, backend="hip", return_w=True, algo=TWO, checkpoint=ck, checkpoint_every=200, chunk=8)
    assert full.iters == 546 and os.path.exists(ck + ".r0")
    res = solve(prob, backend="hip", return_w=True, algo=TWO, resume=ck, chunk=8)
    assert res.converged and res.iters == full.iters
    assert np.array_equal(res.w, full.w)
    with pytest.raises(RuntimeError, match="has the two-step layout.*pass --algo two-step"):  # not resumable here
        solve(prob, backend="hip", algo="fused", resume=ck)


def test_two_step_breakdown_and_nonfinite(gpu, monkeypatch):
    """zero@iter:20 zeroes the (p, Ap) sums of the sweep completing iteration 20:
    iteration 21 (the next sweep's first) breaks down before its update and w
    is the 20-iteration one; nan@iter stops with a non-finite status."""
    prob = EllipseProblem(200, 300)
    monkeypatch.setenv("PE_FAULT_INJECT", "zero@iter:20")
    brk = solve(prob, backend="hip", return_w=True, algo=TWO)
    assert brk.breakdown and not brk.converged and brk.iters == 21
    monkeypatch.setenv("PE_FAULT_INJECT", "nan@iter:20")
    bad = solve(prob, backend="hip", algo=TWO)
    assert bad.nonfinite and 21 <= bad.iters <= 22
    monkeypatch.delenv("PE_FAULT_INJECT")
    capped = EllipseProblem(200, 300)
    capped.max_iter = 20
    ref = solve(capped, backend="hip", return_w=True, algo=TWO)
    np.testing.assert_array_equal(brk.w, ref.w)


def test_two_step_random_init(gpu):
    prob = EllipseProblem(200, 300)
    c = solve(prob, backend="serial", init="random", seed=11, return_w=True)
    d = solve(prob, backend="hip", init="random", seed=11, return_w=True, algo=TWO)
    assert abs(c.iters - d.iters) <= 1
    np.testing.assert_allclose(d.w, c.w, rtol=0, atol=1e-9)


def test_two_step_rejects_odd_counts(gpu, nat):
    """The two-step sweep has no partial sweep (its one-iteration sweep ends
    the solve): an odd run_iterations count is refused instead of silently
    running one iteration more; even counts run exactly."""
    from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

    prob = EllipseProblem(300, 420)
    opt = nat.SolveOptions()
    opt.algo = 3
    opt.check_tol = False
    s = nat.DeviceSolver(prob.to_native(), D.block(300, 420, 1, 0), None, opt)
    s.reset()
    with pytest.raises(ValueError, match="even number"):
        s.run_iterations(7, False)
    s.run_iterations(8, False)
    s.synchronize()
    assert s.state()["iter"] == 8 and s.state()["status"] == 0

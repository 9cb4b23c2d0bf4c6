"""The PyTorch fp64 oracle vs the native CPU backend, and the kernels'
on-the-fly coefficient path (chord tables + per-row classes, host mirror)
vs the oracle's fic_reg assembly — bit-for-bit."""

import numpy as np
import pytest
import torch

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve
from poisson_ellipse_openmp_mpi_cuda_amd.ops import torch_ref
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

VARIANTS = [
    (40, 40, {}),
    (400, 600, {}),
    (257, 129, {}),
    (31, 17, {}),
    (1000, 37, {}),
    (512, 512, dict(A2=-1.0, B2=1.0, cy=1.0)),                               # circle
    (300, 200, dict(A1=-2.0, B1=2.0, A2=-1.0, B2=1.0, cx=0.25, cy=1.0)),     # wide ellipse
]


@pytest.mark.parametrize("M,N,kw", VARIANTS)
def test_coefficient_classes_bitwise(nat, M, N, kw):
    prob = EllipseProblem(M, N, **kw)
    a_t, b_t, _ = torch_ref.assemble(prob)
    a_t, b_t = a_t.numpy(), b_t.numpy()
    counts = np.zeros(3, dtype=np.int64)
    for P in (1, 3, 4, 7):
        for r in range(P):
            blk = D.block(M, N, P, r)
            a, b, c = nat.host_coefficients(prob.to_native(), blk)
            i0, j0 = blk.i0 - 1, blk.j0 - 1
            sl = (slice(i0, i0 + blk.nx + 2), slice(j0, j0 + blk.ny + 2))
            assert np.array_equal(np.asarray(a), a_t[sl])
            assert np.array_equal(np.asarray(b), b_t[sl])
            counts += np.bincount(np.asarray(c).ravel(), minlength=3)
    # on real grids the boundary band (class 2) is a small fraction of all nodes
    if min(M, N) >= 100:
        assert counts[2] < 0.1 * counts.sum()


@pytest.mark.parametrize("M,N,norm", [(40, 40, "weighted"), (60, 90, "weighted"), (40, 40, "unweighted")])
def test_torch_pcg_matches_native(M, N, norm):
    prob = EllipseProblem(M, N, norm=norm)
    nat_rep = solve(prob, backend="serial", return_w=True)
    r = torch_ref.pcg(prob)
    assert abs(r.iters - nat_rep.iters) <= 1
    np.testing.assert_allclose(r.w[1:-1, 1:-1].numpy(), nat_rep.w, rtol=0, atol=1e-9)
    assert r.l2_err == pytest.approx(nat_rep.l2_err, rel=1e-6)


def test_operator_symmetric_positive():
    prob = EllipseProblem(24, 18)
    a, b, _ = torch_ref.assemble(prob)
    g = torch.Generator().manual_seed(0)
    u = torch.rand(prob.M + 1, prob.N + 1, dtype=torch.float64, generator=g)
    v = torch.rand(prob.M + 1, prob.N + 1, dtype=torch.float64, generator=g)
    for t in (u, v):
        t[0, :] = t[-1, :] = 0
        t[:, 0] = t[:, -1] = 0
    Au = torch_ref.apply_A(u, a, b, prob.h1, prob.h2)
    Av = torch_ref.apply_A(v, a, b, prob.h1, prob.h2)
    lhs = torch_ref.dot(Au, v, prob.h1, prob.h2)
    rhs = torch_ref.dot(u, Av, prob.h1, prob.h2)
    assert lhs == pytest.approx(rhs, rel=1e-10)
    assert torch_ref.dot(Au, u, prob.h1, prob.h2) > 0


@pytest.mark.parametrize("M,N", [(40, 40), (60, 90), (31, 17)])
def test_two_step_recurrence_is_pcg(M, N):
    """The two-iterations-per-sweep recurrence of csrc/hip/fused2.hip
    (torch_ref.two_step: scalars of iterations K+1, K+2 from 20 dot products
    of the basis around r_K, p_K) against the reference PCG and the single-sweep
    recurrence: same α, β, w to rounding, and the same stop iteration."""
    prob = EllipseProblem(M, N)
    J = 12
    two = torch_ref.two_step(prob, J)
    one = torch_ref.single_sweep(prob, 2 * J)
    for j in range(J):
        for s in range(2):
            assert two.alpha[j][s] == pytest.approx(one.alpha[2 * j + s], rel=1e-10)
            assert two.beta[j][s] == pytest.approx(one.beta[2 * j + s], rel=1e-9, abs=1e-14)
    scale = float(one.w.abs().max())
    assert float((two.w - one.w).abs().max()) <= 1e-12 * scale
    # iteration count of the reference loop: the first k with ‖Δw‖ < δ
    ref = torch_ref.pcg(prob)
    diffs = [d for pair in two.diff for d in pair]
    k = next((i + 1 for i, d in enumerate(diffs) if d < prob.tol), None)
    if k is not None:
        assert k == ref.iters


def test_two_step_stop_test_matches_reference_history():
    """‖Δw‖ of every iteration from the 20-sum quadratic forms equals the
    reference loop's directly computed norm (rel 1e-7) up to convergence."""
    prob = EllipseProblem(40, 40)
    ref = torch_ref.pcg(prob, keep_history=True)
    two = torch_ref.two_step(prob, (ref.iters + 1) // 2)
    diffs = [d for pair in two.diff for d in pair][: ref.iters]
    np.testing.assert_allclose(diffs, ref.history, rtol=1e-7)


@pytest.mark.parametrize("M,N", [(40, 40), (60, 90), (31, 17)])
def test_three_step_recurrence_is_pcg(M, N):
    """The three-iterations-per-sweep recurrence of csrc/hip/fused3.hip
    (torch_ref.three_step: scalars of iterations K+1..K+3 from 16 D-moments of
    z, p around r_K, p_K) against the single-sweep recurrence: same α, β, w to
    rounding; its late ‖Δw‖ gives the reference's stop iteration."""
    prob = EllipseProblem(M, N)
    J = 8
    three = torch_ref.three_step(prob, J)
    one = torch_ref.single_sweep(prob, 3 * J)
    for j in range(J):
        for s in range(3):
            assert three.alpha[j][s] == pytest.approx(one.alpha[3 * j + s], rel=1e-9)
            assert three.beta[j][s] == pytest.approx(one.beta[3 * j + s], rel=1e-8, abs=1e-14)
    scale = float(one.w.abs().max())
    assert float((three.w - one.w).abs().max()) <= 1e-11 * scale
    ref = torch_ref.pcg(prob)
    diffs = [d for t in three.diff for d in t]
    k = next((i + 1 for i, d in enumerate(diffs) if d < prob.tol), None)
    if k is not None:
        assert k == ref.iters


def test_three_step_stop_test_matches_reference_history():
    """‖Δw‖ of every iteration from the three-step sweep's own ‖p_i‖² sums
    equals the reference loop's norm (rel 1e-7) up to convergence."""
    prob = EllipseProblem(40, 40)
    ref = torch_ref.pcg(prob, keep_history=True)
    three = torch_ref.three_step(prob, (ref.iters + 2) // 3)
    diffs = [d for t in three.diff for d in t][: ref.iters]
    np.testing.assert_allclose(diffs, ref.history, rtol=1e-7)

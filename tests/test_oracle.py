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

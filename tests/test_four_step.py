"""MI355X tests of the four-step sweep (csrc/hip/fused4.hip, opt-in:
--algo four-step / PE_STEPS=4): FOUR Jacobi-PCG iterations per launch from
26 moment sums of the previous sweep (s = 4 moment form, 8-deep halo, one
wave per SIMD).  The moment form is checked against the reference's own
iteration counts (golden values; every count here stops inside a sweep —
546, 1858, 1730 ≡ 2 and 989 ≡ 1 mod 4 — so the late stop test, the w
fix-up and the replay of the last sweep all run), against the
end-of-solve true residual, and across virtual ranks and the iteration cap.
Numerics of s = 4 before any kernel: tools/sstep_proto.py 4,
profiles/r5_sstep4.txt."""

import numpy as np
import pytest

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, solve
from poisson_ellipse_openmp_mpi_cuda_amd.models.ellipse import GOLDEN_ITERS, GOLDEN_L2

pytestmark = pytest.mark.gpu
FOUR = "four-step"


@pytest.mark.parametrize("M,N", [(400, 600), (800, 1200), (1600, 2400), (2048, 2048)])
def test_four_step_golden(gpu, M, N):
    rep = solve(EllipseProblem(M, N), backend="hip", algo=FOUR)
    assert rep.algo == FOUR and rep.converged
    assert rep.iters == GOLDEN_ITERS[(M, N, "weighted")]
    assert rep.l2_err == pytest.approx(GOLDEN_L2[(M, N)], rel=5e-3)
    # the moment recurrence's r is B - A w of the returned iterate
    assert 0 <= rep.res_gap < 1e-4 and rep.restarts == 0


def test_four_step_matches_three_step_w(gpu):
    prob = EllipseProblem(1600, 2400)
    a = solve(prob, backend="hip", algo="three-step", return_w=True)
    b = solve(prob, backend="hip", algo=FOUR, return_w=True)
    assert a.iters == b.iters
    np.testing.assert_allclose(b.w, a.w, rtol=0, atol=1e-9 * np.abs(a.w).max())


@pytest.mark.parametrize("cap", [7, 9, 12])
def test_four_step_iteration_cap(gpu, cap):
    """A cap that is not a multiple of 4 ends with a partial sweep; the w of
    the capped solve equals the three-step sweep's."""
    prob = EllipseProblem(400, 600)
    prob.max_iter = cap
    a = solve(prob, backend="hip", algo="three-step", return_w=True)
    b = solve(prob, backend="hip", algo=FOUR, return_w=True)
    assert a.iters == b.iters == cap and not b.converged
    np.testing.assert_allclose(b.w, a.w, rtol=0, atol=1e-9 * max(1e-30, np.abs(a.w).max()))


@pytest.mark.parametrize("ranks,decomp", [(3, "rows"), (4, "2x2")])
def test_four_step_virtual_ranks(gpu, monkeypatch, ranks, decomp):
    """Virtual ranks on one GPU (the group driver exchanges the 8-deep halos
    and sums the 26 moment sums of every sweep)."""
    monkeypatch.setenv("PE_STEPS", "4")
    prob = EllipseProblem(400, 600)
    one = solve(prob, backend="hip", algo=FOUR, return_w=True)
    grp = solve(prob, backend="hip-group", ranks=ranks, decomp=decomp, return_w=True)
    assert grp.algo == FOUR and grp.iters == one.iters == 546
    np.testing.assert_allclose(grp.w, one.w, rtol=0, atol=1e-9)


def test_four_step_random_init_vs_single_sweep(gpu):
    prob = EllipseProblem(2048, 2048)
    four = solve(prob, backend="hip", algo=FOUR, init="random", seed=1234, return_w=True)
    one = solve(prob, backend="hip", algo="fused", init="random", seed=1234, return_w=True)
    assert four.converged and one.converged and abs(four.iters - one.iters) <= 1
    assert np.abs(four.w - one.w).max() <= 1e-7 * np.abs(one.w).max()
    assert four.res_gap < 1e-4

"""MI355X tests of the static item layouts (csrc/hip/item_layout.cpp): every
owned row of every strip is marched exactly once, whatever the layout — the
three-step filling layout (kind-aware costs, items cut to fill each wave),
the equal-cost layout (PE_LAYOUT=equal), the LPT layout (PE_LAYOUT=lpt) and
the overlap's boundary-first order — and the equal-cost layout evens the
waves' estimated loads.  Construction only (no solve)."""

import numpy as np
import pytest

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D

pytestmark = pytest.mark.gpu
BAND, UNI = 1 << 30, 1 << 29


def _coverage(s, nx, ny):
    ent = [e for e in s.layout_entries if e[1] > 0]
    nstrips = s.strips
    assert nstrips == (ny + 47) // 48  # 48 output columns per three-step strip (fused3.hip)
    cov = np.zeros((nstrips, nx + 1), dtype=np.int32)
    for ib, rows, strip, _flags in ent:
        assert 0 <= strip < nstrips and ib >= 1 and ib + rows - 1 <= nx
        cov[strip, ib:ib + rows] += 1
    assert (cov[:, 1:] == 1).all(), "a row of a strip is marched twice or never"
    return ent


@pytest.mark.parametrize("P,spec,env", [(1, "device", {}), (1, "device", {"PE_LAYOUT": "equal"}),
                                        (1, "device", {"PE_LAYOUT": "fill"}), (8, "device", {}),
                                        (2, "device", {}), (4, "device", {"PE_LAYOUT": "equal"}),
                                        (8, "4x2", {"PE_OVERLAP": "1"})])
def test_layout_covers_every_row_once(gpu, nat, monkeypatch, P, spec, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    M = N = 8192
    g = D.grid(P, M, N, spec)
    blk = nat.decompose(M, N, g, P // 2)
    opt = nat.SolveOptions()
    opt.check_tol = False
    comm = nat.make_delay_comm(P, 0.0, 0.0) if P > 1 else None
    s = nat.DeviceSolver(EllipseProblem(M, N).to_native(), blk, comm, opt)
    assert s.sweep_steps == 3
    _coverage(s, blk.nx, blk.ny)
    mx, mean, per = s.layout_load
    if s.layout_name == "equal" and env.get("PE_OVERLAP") != "1":
        # exactly k pieces per wave, estimated loads within a few percent (with
        # the overlap, the 6-row boundary pieces cut off for the exchange are
        # a wave's whole share on small blocks: no balance bound there)
        assert mx <= 1.08 * mean, (mx, mean)
        ent = [e for e in s.layout_entries if e[1] > 0]
        assert (per - 1) * s.layout_waves < len(ent) <= per * s.layout_waves

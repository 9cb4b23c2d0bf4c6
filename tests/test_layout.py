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


def _boundary_first(s, blk):
    """Overlap: the kernel's kSignal variant counts list positions 0 .. nb-1
    as the boundary items (outputs a neighbour needs: the 6 owned rows /
    columns next to it) and starts the exchange when they are stored — so
    those positions hold exactly the boundary items."""
    nb = s.layout_boundary
    assert nb > 0
    nx, ny = blk.nx, blk.ny
    has = [blk.nbr[i] >= 0 for i in range(4)]  # LEFT, RIGHT, DOWN, UP

    def bnd(ib, rows, strip):
        j0 = -7 + 48 * strip
        jlo, jhi = max(1, j0 + 8), min(ny, j0 + 55)
        return ((has[0] and ib <= 6) or (has[1] and ib + rows - 1 >= nx - 5) or (has[2] and jlo <= 6)
                or (has[3] and jhi >= ny - 5))

    ents = s.layout_entries
    for pos, (ib, rows, strip, _flags) in enumerate(ents):
        if rows == 0:
            continue
        assert bnd(ib, rows, strip) == (pos < nb), (pos, nb, ib, rows, strip)


@pytest.mark.parametrize("P,spec,env", [(1, "device", {}), (1, "device", {"PE_LAYOUT": "equal"}),
                                        (1, "device", {"PE_LAYOUT": "fill"}), (8, "device", {}),
                                        (2, "device", {}), (4, "device", {"PE_LAYOUT": "equal"}),
                                        (8, "4x2", {"PE_OVERLAP": "1"}), (6, "2x3", {"PE_OVERLAP": "1"}),
                                        (4, "2x2", {"PE_OVERLAP": "1", "PE_LAYOUT": "lpt"}),
                                        (8, "device", {"PE_YOUNG": "1.25"}), (1, "device", {"PE_YOUNG": "1.25"})])
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
    ent = _coverage(s, blk.nx, blk.ny)
    if env.get("PE_OVERLAP") == "1":
        _boundary_first(s, blk)
    mx, mean, per = s.layout_load
    if s.layout_name == "equal" and env.get("PE_OVERLAP") != "1":
        # exactly k pieces per wave, estimated loads within a few percent (with
        # the overlap, the 6-row boundary pieces cut off for the exchange are
        # a wave's whole share on small blocks: no balance bound there)
        assert mx <= 1.10 * mean, (mx, mean)  # (8192² at 112 rows: 7 pieces per wave, 1.09)
        ent = [e for e in s.layout_entries if e[1] > 0]
        assert (per - 1) * s.layout_waves < len(ent) <= per * s.layout_waves


def test_overlap_full_grid_launches(gpu, nat, monkeypatch):
    """Launches that use the whole grid (S_0, the construction's timing
    sweeps, the replay) include the overlap's reserved blocks: their waves
    have no list positions (they used to march round r+1's first items a
    second time, so S_0 counted those items' sums twice).  One rank's 4x2
    block of 8192² (two rounds of items): 30 iterations with the overlap
    give the w of 30 without it, to rounding (the boundary-first order sums
    in another order)."""
    g = D.grid(8, 8192, 8192, "4x2")
    blk = nat.decompose(8192, 8192, g, 4)
    monkeypatch.setenv("PE_TI", "48")  # (fixed rows per item: two rounds of LPT items)
    monkeypatch.setenv("PE_LAYOUT", "lpt")
    ws = []
    for ov in ("0", "1"):
        monkeypatch.setenv("PE_OVERLAP", ov)
        opt = nat.SolveOptions()
        opt.check_tol = False
        comm = nat.make_delay_comm(8, 0.0, 0.0)
        s = nat.DeviceSolver(EllipseProblem(8192, 8192).to_native(), blk, comm, opt)
        if ov == "1":
            assert s.layout_boundary > 0 and len([e for e in s.layout_entries if e[1] > 0]) > s.layout_waves
        s.reset()
        s.run_iterations(30, False)
        s.synchronize()
        ws.append(np.array(s.w()))
        del s, comm
    scale = np.abs(ws[0]).max()
    assert scale > 0 and np.abs(ws[0] - ws[1]).max() <= 1e-9 * scale


def test_priority_turns_and_wave_map_keep_the_sums(gpu, nat, monkeypatch):
    """SIMD priority turns (PE_PRIO, fused3.hip prio_turn) change only when
    waves issue: 30 iterations give the same bits with and without them, and
    with and without the first rows staged into LDS (PE_STAGE).  A
    permuted list -> workgroup map (PE_WPERM) groups other items into each
    workgroup's partial sum: the same w to rounding.  2048² on one GPU, fixed
    rows per item (no timing-dependent tuning)."""
    monkeypatch.setenv("PE_TI", "64")
    monkeypatch.setenv("PE_LAYOUT", "equal")
    ws = {}
    for name, env in (("off", {"PE_PRIO": "0"}), ("turns", {"PE_PRIO": "10"}), ("fast", {"PE_PRIO": "7"}),
                      ("nostage", {"PE_PRIO": "0", "PE_STAGE": "0"}),
                      ("perm", {"PE_PRIO": "0", "PE_WPERM": "1"})):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        blk = nat.decompose(2048, 2048, D.grid(1, 2048, 2048, "device"), 0)
        opt = nat.SolveOptions()
        opt.check_tol = False
        s = nat.DeviceSolver(EllipseProblem(2048, 2048).to_native(), blk, None, opt)
        assert s.sweep_steps == 3 and not s.resident
        s.reset()
        s.run_iterations(30, False)
        s.synchronize()
        ws[name] = np.array(s.w())
        del s
        monkeypatch.delenv("PE_WPERM", raising=False)
        monkeypatch.delenv("PE_STAGE", raising=False)
    scale = np.abs(ws["off"]).max()
    assert scale > 0
    assert np.array_equal(ws["off"], ws["turns"]) and np.array_equal(ws["off"], ws["fast"])
    # the first rows staged into LDS at kernel entry (default) or loaded by the march (PE_STAGE=0): same bits
    assert np.array_equal(ws["off"], ws["nostage"])
    assert np.abs(ws["off"] - ws["perm"]).max() <= 1e-9 * scale


@pytest.mark.parametrize("M,N", [(2048, 2048), (2400, 3200)])
def test_tuned_layout_is_a_fresh_layout(gpu, nat, monkeypatch, M, N):
    """The rows-per-item tuning runs its trials pipelined and ends on a layout
    from its cache (the finalists', the final one; the equal-cost layout's
    runs are cached too): that list is the one a fresh construction builds at
    the same height and layout, entry for entry."""
    for k in ("PE_TI", "PE_LAYOUT", "PE_TI_TUNE"):
        monkeypatch.delenv(k, raising=False)
    prob = EllipseProblem(M, N).to_native()
    blk = D.block(M, N, 1, 0)
    s1 = nat.DeviceSolver(prob, blk, None, nat.SolveOptions())
    assert len(s1.ti_tuning_ms) > 0
    ti, lay, ent1 = s1.ti, s1.layout_name, [tuple(e) for e in s1.layout_entries]
    del s1
    monkeypatch.setenv("PE_TI", str(ti))
    monkeypatch.setenv("PE_LAYOUT", lay)
    s2 = nat.DeviceSolver(prob, blk, None, nat.SolveOptions())
    assert len(s2.ti_tuning_ms) == 0 and s2.ti == ti and s2.layout_name == lay
    assert [tuple(e) for e in s2.layout_entries] == ent1


def test_halo_choice_layout_is_a_fresh_layout(gpu, nat, monkeypatch):
    """The halo-path choice switches between cached layouts (the overlap at the
    tuning's three best heights); the overlapped list it ends on is the one a
    fresh construction lays out at that height, entry for entry.  One rank's
    block of the 8-rank slab of 8192², delay transport, the exchange's overlap
    forced (PE_HALO=exchange PE_OVERLAP=1)."""
    M = N = 8192
    prob = EllipseProblem(M, N).to_native()
    blk = nat.decompose(M, N, D.grid(8, M, N, "rows"), 4)
    for k in ("PE_TI", "PE_LAYOUT", "PE_HALO_TUNE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("PE_HALO", "exchange")
    monkeypatch.setenv("PE_OVERLAP", "1")
    opt = nat.SolveOptions()
    opt.check_tol = False
    c1 = nat.make_delay_comm(8, 0.0, 0.0, True)
    s1 = nat.DeviceSolver(prob, blk, c1, opt)
    assert s1.overlap and s1.halo_path == "exchange+overlap"
    assert len([n for n, _ in s1.halo_candidates if "(again)" not in n]) >= 2  # (several heights timed)
    ti, ent1, nb1 = s1.ti, [tuple(e) for e in s1.layout_entries], s1.layout_boundary
    del s1, c1
    monkeypatch.setenv("PE_TI", str(ti))
    c2 = nat.make_delay_comm(8, 0.0, 0.0, True)
    s2 = nat.DeviceSolver(prob, blk, c2, opt)
    assert s2.overlap and s2.ti == ti
    assert s2.layout_boundary == nb1
    assert [tuple(e) for e in s2.layout_entries] == ent1

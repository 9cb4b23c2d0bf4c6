"""Sweep timeline of the single-sweep kernel from in-kernel stamps.

One GPU runs the block of one rank of a P-rank decomposition of 8192²
(timing-only transport, zero delays, overlap off), with PE_STAMPS=1: a
diagnostic build of the sweep writes, per work item, s_memrealtime at its
start and end (100 MHz) and, per wave, its entry and exit.  The last sweep's
stamps are read back and summarised: kernel span, wave entry spread, first
item latency, item duration distribution, gaps between a wave's items, and
the tail (how long the chip runs partly idle at the end).  The stamped
build's own run time is not a measurement of the real kernel: read shares.

    PROBE_CFG=8:aspect,1:aspect PROBE_ENV="PE_TI=8;PE_TI=16" python tools/stamp_probe.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PE_STAMPS"] = "1"
os.environ["PE_OVERLAP"] = "0"

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402


def pct(a, q):
    return float(np.percentile(a, q)) if len(a) else float("nan")


def step_timeline(steps: np.ndarray, three: bool = False) -> str:
    """Median time (µs) from a wave's first item start to each stamped point of that item."""
    s = steps.reshape(-1, 32).astype(np.int64)
    s = s[s[:, 0] > 0]
    if not len(s):
        return "  (no step stamps)"
    if three:  # fused3.hip kStamp: [1] kernel entry, [2] prologue issued, [3..30] after each 6-step group, [31] end
        names = {1: "kernel entry (wave)", 2: "prologue issued", 31: "item end"}
        names.update({c: f"after row step {6 * (c - 2):d}" for c in range(3, 31)})
    else:
        names = {1: "prologue issued", 2: "row classes in", 3: "prologue rows in", 31: "item end"}
    out = ["  first-item timeline (median us after item start, n waves; per-group increment):"]
    prev = None
    for c in range(1, 32):
        if three and c >= 24 and c <= 30:  # (24-27: prologue points, 28/29: shader clock, 30: hardware id)
            continue
        v = s[:, c]
        ok = v > 0
        if ok.sum() < max(1, len(s) // 4):
            continue
        d = (v[ok] - s[ok, 0]) / 100.0
        med = float(np.median(d))
        inc = "" if prev is None or c < 3 else f"  +{med - prev:6.2f}"
        out.append(f"    {names.get(c, f'after row step {c - 6:+d}'):22s} {med:7.2f}{inc}  (n {ok.sum()})")
        if c >= 2:
            prev = med
    return "\n".join(out)


def grid_timeline(glob: np.ndarray, steps: np.ndarray, wv_all: np.ndarray) -> str:
    """Three-step kStamp: the launch around the item walk — kernel entry, the
    walk, the grid reduction and finalize, and the gap after the previous
    launch's finalize (µs)."""
    s = steps.reshape(-1, 32).astype(np.int64)
    ent = s[:, 1][s[:, 1] > 0]
    g = glob.astype(np.int64)
    if not len(ent) or g[2] == 0:
        return "  (no grid stamps)"
    t0 = ent.min()
    wv = wv_all[wv_all[:, 0] > 0]
    first_items = s[:, 0][s[:, 0] > 0]
    out = ["  launch timeline (us from the first wave's kernel entry):"]
    if g[0] > 0:
        out.append(f"    gap after the previous launch's finalize: {(t0 - g[0]) / 100.0:7.2f}")
    out.append(f"    wave kernel entry: median {np.median(ent - t0) / 100.0:6.2f}  max {(ent.max() - t0) / 100.0:6.2f}")
    for slot, nm in ((24, "state read, stop tests decided"), (25, "step scalars formed")):
        v = s[:, slot][s[:, slot] > 0]
        if len(v):
            out.append(f"    {nm}: median {np.median(v - t0) / 100.0:6.2f}  (after the wave's own entry: "
                       f"{np.median((s[:, slot] - s[:, 1])[s[:, slot] > 0]) / 100.0:5.2f})")
    out.append(f"    walk entry (scalars + ring): median {np.median(wv[:, 0] - t0) / 100.0:6.2f}")
    out.append(f"    first item start: median {np.median(first_items - t0) / 100.0:6.2f}")
    out.append(f"    last wave exit {(wv[:, 1].max() - t0) / 100.0:7.2f}; grid reduction start {(g[1] - t0) / 100.0:7.2f}; "
               f"finalized {(g[2] - t0) / 100.0:7.2f}")
    if g[5] > 0 and g[6] > 0:  # the last block: block reduction, publish, partials summed, finalize start
        out.append(f"    last block: block reduce {(g[5] - t0) / 100.0:7.2f}, publish {(g[6] - t0) / 100.0:7.2f}, ticket won "
                   f"{(g[1] - t0) / 100.0:7.2f}, partials summed {(g[3] - t0) / 100.0:7.2f}, finalize start "
                   f"{(g[4] - t0) / 100.0:7.2f}, done {(g[2] - t0) / 100.0:7.2f}")
    return "\n".join(out)


def simd_tail(steps: np.ndarray, wv_all: np.ndarray) -> str:
    """Three-step kStamp: slot 30 holds the wave's HW_ID | XCC_ID << 32 — the
    exits per SIMD (the last of its waves) and per CU: is the tail whole
    SIMDs idle, or a SIMD running one wave instead of two?"""
    s = steps.reshape(-1, 32).astype(np.int64)
    hw = s[:, 30]
    live = (wv_all[: len(hw), 0] > 0) & (s[:, 1] > 0)
    if not live.any():
        return "  (no hardware ids)"
    hw, ex = hw[live], wv_all[: len(live)][live, 1]
    t0 = s[live, 1].min()
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = (hw >> 32) & 15
    cuk = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    simdk = cuk * 4 + simd
    out = [f"  placement: {len(np.unique(cuk))} CUs, {len(np.unique(simdk))} SIMDs, {len(np.unique(xcc))} XCCs; "
           f"waves per SIMD max {np.bincount(np.unique(simdk, return_inverse=True)[1]).max()}"]
    for name, key in (("SIMD", simdk), ("CU", cuk)):
        u, inv = np.unique(key, return_inverse=True)
        last = np.zeros(len(u), dtype=np.int64)
        np.maximum.at(last, inv, ex)
        e = (last - t0) / 100.0
        out.append(f"  {name} exit (its last wave): min {e.min():6.1f} p10 {pct(e, 10):6.1f} median {np.median(e):6.1f} "
                   f"p90 {pct(e, 90):6.1f} max {e.max():6.1f} us")
    # per SIMD: first and last wave exit (one wave alone for how long)
    u, inv = np.unique(simdk, return_inverse=True)
    first = np.full(len(u), np.iinfo(np.int64).max)
    last = np.zeros(len(u), dtype=np.int64)
    np.minimum.at(first, inv, ex)
    np.maximum.at(last, inv, ex)
    alone = (last - first) / 100.0
    out.append(f"  SIMD with one wave left: median {np.median(alone):6.1f} p90 {pct(alone, 90):6.1f} us (last minus first wave exit)")
    # shader clock over each wave's life: Δ s_memtime (cycles) / Δ s_memrealtime (100 MHz)
    mt0, mt1 = s[live, 28], s[live, 29]
    rt0, rt1 = s[live, 1], wv_all[: len(live)][live, 1]
    ok = (mt1 > mt0) & (rt1 > rt0 + 1000)
    if ok.any():
        ghz = (mt1[ok] - mt0[ok]) / ((rt1[ok] - rt0[ok]) * 10.0)  # cycles per 10 ns tick -> GHz
        out.append(f"  shader clock over a wave's life: median {np.median(ghz):5.3f} GHz  p10 {pct(ghz, 10):5.3f}  p90 {pct(ghz, 90):5.3f}"
                   f"  (by XCC: {' '.join(f'{np.median(ghz[xcc[ok] == x]):.2f}' for x in range(8) if (xcc[ok] == x).any())})")
    return "\n".join(out)


def summarise(st: np.ndarray, nitems: int, nw: int, three: bool = False) -> str:
    steps = st[len(st) - 32 * nw:]
    glob = st[len(st) - 32 * nw - 8: len(st) - 32 * nw]
    st = st[: len(st) - 32 * nw]
    nslots = nitems
    it = st[: 4 * nslots].reshape(nslots, 4).astype(np.int64)
    it = it[it[:, 0] > 0]  # static layouts have empty positions
    nitems = len(it)
    geo = it[:, 3].copy()
    strip = it[:, 2] >> 32
    it[:, 2] &= 0xFFFFFFFF  # wave id
    wv_all = st[4 * nslots : 4 * nslots + 2 * nw].reshape(-1, 2).astype(np.int64)
    live = wv_all[:, 0] > 0
    wv = wv_all[live]
    t0 = wv[:, 0].min()
    us = lambda x: x / 100.0  # 100 MHz ticks → µs  # noqa: E731
    end = max(wv[:, 1].max(), it[:, 1].max())
    span = us(end - t0)
    dur = us(it[:, 1] - it[:, 0])
    out = [f"  span {span:7.1f} us  waves {len(wv)}  items {nitems}  items/wave {nitems / len(wv):.1f}"]
    ent = us(wv[:, 0] - t0)
    out.append(f"  wave entry after the first: median {np.median(ent):6.1f}  p99 {pct(ent, 99):6.1f}  max {ent.max():6.1f} us")
    ex = us(wv[:, 1] - t0)
    out.append(f"  wave exit: min {ex.min():6.1f}  p10 {pct(ex, 10):6.1f}  median {np.median(ex):6.1f}  max {ex.max():6.1f} us"
               f"  -> tail (max - median) {ex.max() - np.median(ex):5.1f} us")
    med = np.median(dur)
    out.append(f"  item duration: p10 {pct(dur, 10):6.2f}  median {med:6.2f}  p90 {pct(dur, 90):6.2f}"
               f"  p99 {pct(dur, 99):6.2f}  max {dur.max():6.2f} us")
    slow = dur > 1.5 * med
    out.append(f"  items > 1.5x median: {slow.sum()} ({100 * slow.mean():.1f} %), {100 * dur[slow].sum() / dur.sum():.1f} % of item time")
    order = np.lexsort((it[:, 0], it[:, 2]))
    first_lat, gaps = [], []
    prev_w, prev_end = -1, 0
    for s0, s1, w, _b in it[order]:
        if w != prev_w:
            if 0 <= w < len(wv_all) and wv_all[w, 0] > 0:
                first_lat.append(us(s0 - wv_all[w, 0]))
            prev_w = w
        else:
            gaps.append(us(s0 - prev_end))
        prev_end = s1
    out.append(f"  first item start after wave entry: median {np.median(first_lat):6.2f}  p90 {pct(first_lat, 90):6.2f} us")
    if gaps:
        out.append(f"  gap between a wave's items: median {np.median(gaps):6.3f}  p90 {pct(gaps, 90):6.3f} us")
    # time profile of busy waves (10 bins)
    edges = np.linspace(t0, end, 11)
    prof = []
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(it[:, 1], b) - np.maximum(it[:, 0], a), 0, None).sum()
        prof.append(ov / ((b - a) * len(wv)))
    out.append("  busy waves per tenth of the span: " + " ".join(f"{p:4.2f}" for p in prof))
    out.append(f"  busy fraction (item time / waves x span) {dur.sum() / (len(wv) * span):5.3f}")
    late = np.argsort(it[:, 1])[-8:]
    for i in late:
        out.append(f"    late item: start {us(it[i, 0] - t0):6.1f} end {us(it[i, 1] - t0):6.1f} us  rows {geo[i] & 0xFFFFFFFF}"
                   f"+{(geo[i] >> 32) & 0xFFFF}  strip {strip[i]}  band {geo[i] >> 48}  wave {it[i, 2]}")
    band = (geo >> 48) == 1
    if band.any():
        out.append(f"  band items: {band.sum()}  duration median {np.median(dur[band]):6.2f} us; others {np.median(dur[~band]):6.2f} us")
    # per item kind (three-step sweep: 0 mixed, 1 band, 2 uniform): time per row step
    # of the march (rows + 2*halo fill steps) -> the layout's cost model
    rows = (geo >> 32) & 0xFFFF
    kind = geo >> 48
    halo = int(os.environ.get("PROBE_HALO", "6"))
    for kd, name in ((2, "uniform"), (0, "mixed"), (1, "band")):
        m = kind == kd
        if m.any():
            per = dur[m] / (rows[m] + 2 * halo)
            # least squares dur = a * steps + b
            A = np.stack([rows[m] + 2 * halo, np.ones(m.sum())], 1).astype(float)
            coef = np.linalg.lstsq(A, dur[m], rcond=None)[0] if m.sum() > 2 else (float("nan"), float("nan"))
            out.append(f"  kind {name:7s}: {m.sum():6d} items  us per row step median {np.median(per):6.3f} p90 {pct(per, 90):6.3f}"
                       f"  fit {coef[0]:6.3f} us/step + {coef[1]:6.2f} us")
    wl_all = np.zeros(int(it[:, 2].max()) + 1)
    np.add.at(wl_all, it[:, 2], dur)
    wl = wl_all[wl_all > 0]
    out.append(f"  wave item time: max {wl.max():7.1f}  mean {wl.mean():7.1f}  = {wl.max() / wl.mean():5.3f};"
               f" p10 {pct(wl, 10):7.1f} p90 {pct(wl, 90):7.1f} us")
    # per XCD (workgroup b runs on XCD b mod 8) and per wave slot in the workgroup:
    # item time per row step of the uniform items (the same work everywhere)
    gw = it[:, 2]
    uni = kind == 2
    if uni.any():
        steps_u = (rows + 2 * halo).astype(float)
        per_step = dur / steps_u
        xcd = (gw // 4) % 8
        slot = gw % 4
        out.append("  uniform us/step by XCD: " + " ".join(f"{np.median(per_step[uni & (xcd == x)]):.3f}" for x in range(8)))
        out.append("  uniform us/step by wave slot: " + " ".join(f"{np.median(per_step[uni & (slot == x)]):.3f}" for x in range(4)))
        # by the item's first row (deciles of the block) and by its physical workgroup (deciles of the grid):
        # a position effect (memory) follows the rows under a permuted wave map (PE_WPERM), a hardware one the waves
        r0 = geo & 0xFFFFFFFF
        rb = np.minimum(9, (r0 * 10) // max(1, int(r0.max()) + 1))
        out.append("  uniform us/step by row decile: " + " ".join(f"{np.median(per_step[uni & (rb == x)]):.3f}"
                                                              if (uni & (rb == x)).any() else "  -  " for x in range(10)))
        nwg = int(gw.max()) // 4 + 1
        bb = np.minimum(9, ((gw // 4) * 10) // nwg)
        out.append("  uniform us/step by workgroup decile: " + " ".join(f"{np.median(per_step[uni & (bb == x)]):.3f}"
                                                                    if (uni & (bb == x)).any() else "  -  " for x in range(10)))
        sb = np.minimum(9, (strip * 10) // max(1, int(strip.max()) + 1))
        out.append("  uniform us/step by strip decile: " + " ".join(f"{np.median(per_step[uni & (sb == x)]):.3f}"
                                                                for x in range(10) if (uni & (sb == x)).any()))
        # position in the wave's list (round): early rounds run with the whole chip busy
        rnd = np.zeros(len(it), dtype=int)
        order = np.lexsort((it[:, 0], gw))
        prev = -1
        r = 0
        for i in order:
            r = r + 1 if gw[i] == prev else 0
            prev = gw[i]
            rnd[i] = r
        out.append("  uniform us/step by round: " + " ".join(f"{np.median(per_step[uni & (rnd == x)]):.3f}"
                                                          for x in range(int(rnd.max()) + 1) if (uni & (rnd == x)).any()))
        # a wave's total time against its static cost (row steps, band x2.45): the unexplained spread
        cost = np.where(kind == 1, 2.45, np.where(kind == 0, 1.3, 1.0)) * steps_u
        wc = np.zeros_like(wl_all)
        np.add.at(wc, gw, cost)
        m = wl_all > 0
        ratio = wl_all[m] / wc[m]
        out.append(f"  wave time / static cost: p10 {pct(ratio, 10):.3f} median {np.median(ratio):.3f} p90 {pct(ratio, 90):.3f}"
                   f"  (corr of wave time with cost {np.corrcoef(wl_all[m], wc[m])[0, 1]:.2f})")
    if three:
        out.append(simd_tail(steps, wv_all))
    out.append(step_timeline(steps, three))
    if three:
        out.append(grid_timeline(glob, steps, wv_all))
    return "\n".join(out)


def item_times(st: np.ndarray, nitems: int, nw: int):
    """Per item slot: duration (µs, 0 for an empty slot) and wave; per wave: exit time after the first entry."""
    body = st[: len(st) - 32 * nw - 8]
    it = body[: 4 * nitems].reshape(nitems, 4).astype(np.int64)
    wv = body[4 * nitems: 4 * nitems + 2 * nw].reshape(-1, 2).astype(np.int64)
    dur = np.where(it[:, 0] > 0, (it[:, 1] - it[:, 0]) / 100.0, 0.0)
    live = wv[:, 0] > 0
    ex = np.where(live, (wv[:, 1] - wv[live, 0].min()) / 100.0, np.nan)
    return dur, ex


def persistence(durs) -> str:
    """Is a slow item (or wave) slow again in the next sweep?  Correlations of
    per-item durations and per-wave exit times between consecutive sweeps of
    one process (same layout, same memory): high values would let a layout be
    rebalanced from measured times; low values mean the spread is noise."""
    out = ["  persistence across sweeps (consecutive pairs):"]
    for a in range(len(durs) - 1):
        (d0, e0), (d1, e1) = durs[a], durs[a + 1]
        m = (d0 > 0) & (d1 > 0)
        w = np.isfinite(e0) & np.isfinite(e1)
        # relative duration: item time over the median of its row count is unknown here, use raw
        out.append(f"    sweeps {a}->{a + 1}: item duration corr {np.corrcoef(d0[m], d1[m])[0, 1]:5.2f}  "
                   f"wave exit corr {np.corrcoef(e0[w], e1[w])[0, 1]:5.2f}  "
                   f"late-decile overlap {late_overlap(e0[w], e1[w]):4.2f}")
    e = np.stack([x[1] for x in durs])
    w = np.all(np.isfinite(e), 0)
    mean_ex = e[:, w].mean(0)
    out.append(f"    wave exit averaged over {len(durs)} sweeps: median {np.median(mean_ex):6.1f}  max {mean_ex.max():6.1f}"
               f"  (single sweeps: max - median {np.mean([np.nanmax(x) - np.nanmedian(x) for x in e]):5.1f}; "
               f"averaged: {mean_ex.max() - np.median(mean_ex):5.1f} us)")
    gw = np.nonzero(w)[0]
    xcd = (gw // 4) % 8
    out.append("    mean wave exit by XCD: " + " ".join(f"{np.median(mean_ex[xcd == x]):6.1f}" for x in range(8)))
    return "\n".join(out)


def late_overlap(e0, e1) -> float:
    """Fraction of the last-finishing 10 % of waves in one sweep that are also in the last 10 % of the other."""
    k = max(1, len(e0) // 10)
    a = set(np.argsort(e0)[-k:])
    b = set(np.argsort(e1)[-k:])
    return len(a & b) / k


def main():
    nat = native()
    configs = [(int(c.split(":")[0]), c.split(":")[1]) for c in os.environ.get("PROBE_CFG", "8:aspect,1:aspect").split(",")]
    envs = [e.strip() for e in os.environ.get("PROBE_ENV", "").split(";")]
    GM, GN = (int(v) for v in os.environ.get("PROBE_GRID", "8192x8192").split("x"))
    prob = pe.EllipseProblem(GM, GN)
    for P, spec in configs:
        g = D.grid(P, GM, GN, spec)
        blk = nat.decompose(GM, GN, g, P // 2)
        for env in envs:
            kv = dict(x.split("=") for x in env.split()) if env else {}
            saved = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            opt = nat.SolveOptions()
            opt.check_tol = False
            comm = nat.make_delay_comm(P, 0.0, 0.0) if P > 1 else None
            s = nat.DeviceSolver(prob.to_native(), blk, comm, opt)
            s.reset()
            dt = s.time_iterations(40, False)
            print(f"P={P} {g.Px}x{g.Py} block {blk.nx}x{blk.ny} [{env or 'default'}] ti={s.ti} order={s.order}: "
                  f"{dt / 40 * 1e6:.1f} us/iter (stamped build)", flush=True)
            three = int(s.sweep_steps) >= 3
            s.clear_stamps()
            if three:  # (a launch records the previous one's finalize: the gap between launches)
                s.run_iterations(1, False)
            durs = []
            nrep = int(os.environ.get("PROBE_REPEAT", "2"))
            for rep in range(nrep):  # iterations alternate the two sweep variants
                sweep = ("deferring", "applying")[rep % 2]
                if not three:
                    s.clear_stamps()
                s.run_iterations(1, False)
                st = np.asarray(s.stamps())
                if rep < 2:
                    print(f" one {sweep}-parity sweep:")
                    print(summarise(st, s.nitems, s.stamp_waves, three), flush=True)
                durs.append(item_times(st, s.nitems, s.stamp_waves))
            if nrep > 2:
                print(persistence(durs), flush=True)
            del s, comm
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v


if __name__ == "__main__":
    main()

"""Item-layout knobs compared at ONE memory placement: one solver per block,
re-laid out (DeviceSolver.relayout) for each configuration, then timed.

    PROBE_GRID=8192x8192 PROBE_P=1 PROBE_CFGS="18;18 PE_TAIL_SPLIT=3;18 PE_TAIL_FRAC=0.5" python tools/layout_probe.py

Each configuration: "<rows per item>[s|d] [PE_X=v ...]" (s / d: static LPT
layout / dynamic queue; default: the solver's own); configurations are timed
in rounds (the list repeated PROBE_ROUNDS times) so drift shows.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import poisson_ellipse_openmp_mpi_cuda_amd as pe  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd._loader import native  # noqa: E402
from poisson_ellipse_openmp_mpi_cuda_amd.parallel import decomp as D  # noqa: E402

nat = native()
GM, GN = (int(v) for v in os.environ.get("PROBE_GRID", "8192x8192").split("x"))
P = int(os.environ.get("PROBE_P", "1"))
spec = os.environ.get("PROBE_SPEC", "device")
iters = int(os.environ.get("PROBE_ITERS", "400"))
rounds = int(os.environ.get("PROBE_ROUNDS", "2"))
cfgs = [c.strip() for c in os.environ.get("PROBE_CFGS", "18").split(";") if c.strip()]
prob = pe.EllipseProblem(GM, GN)
os.environ["PE_OVERLAP"] = "0"
g = D.grid(P, GM, GN, spec)
blk = nat.decompose(GM, GN, g, P // 2)
opt = nat.SolveOptions()
opt.check_tol = False
comm = nat.make_delay_comm(P, 0.0, 0.0) if P > 1 else None
s = nat.DeviceSolver(prob.to_native(), blk, comm, opt)
print(f"P={P} block {blk.nx}x{blk.ny}: order {s.order}, placement {[round(x, 4) for x in s.placement_ms]}", flush=True)
for r in range(rounds):
    for c in cfgs:
        parts = c.split()
        kv = dict(x.split("=") for x in parts[1:])
        saved = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        t = parts[0]
        s.relayout(int(t.rstrip("sd")), 0 if t.endswith("s") else 3 if t.endswith("d") else -1)
        s.reset()
        s.time_iterations(20, False)
        dt = s.time_iterations(iters, False)
        mx, mean, per = s.layout_load
        lay = f"  wave load max {mx:.0f} / mean {mean:.0f} = {mx / mean:.3f}, <= {per:.0f} items" if mx else ""
        print(f"  round {r} [{c}]: {dt / iters * 1e6:7.1f} us/iter  order {s.order}  items {s.nitems}{lay}", flush=True)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

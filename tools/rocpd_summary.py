#!/usr/bin/env python3
"""Per-kernel summary and dispatch timeline gaps from a rocprofv3 SQLite
result (`rocprofv3 --kernel-trace -d DIR -o run`).

    python tools/rocpd_summary.py gpurun_out/x/prof/run_results.db [--timeline N] [--segments MS]

--segments MS splits the trace wherever the device idles longer than MS
milliseconds (e.g. between the configurations of tools/block_probe.py) and
prints one table per segment, keyed by kernel and grid size, with medians.
"""
import argparse
import sqlite3
import sys
from collections import defaultdict


def short(n: str) -> str:
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("pe::dev::", "")
    return n.split("(KParams")[0].split("(")[0][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches with gaps")
    ap.add_argument("--skip", type=int, default=0, help="ignore the first N dispatches")
    ap.add_argument("--segments", type=float, default=0.0, help="split at device idle gaps longer than this (ms)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    grid_col = "grid_size_x" if "grid_size_x" in cols else "0"
    rows = list(c.execute(f"select {name_col}, start, end, stream_id, {grid_col} from kernels order by start"))[a.skip:]
    if a.segments > 0:
        segs = [[]]
        prev = None
        for r in rows:
            if prev is not None and r[1] - prev > a.segments * 1e6:
                segs.append([])
            segs[-1].append(r)
            prev = r[2]
        for i, sg in enumerate(segs):
            agg = defaultdict(list)
            for n, s, e, _, g in sg:
                agg[(short(n), g)].append((e - s) / 1e3)
            span = (sg[-1][2] - sg[0][1]) / 1e3
            print(f"segment {i}: {len(sg)} dispatches over {span:.0f} us")
            for (n, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:8]:
                v = sorted(v)
                print(f"   {n:48s} grid {g:8d}  n {len(v):5d}  median {v[len(v) // 2]:9.2f} us  min {v[0]:9.2f} us")
        return 0
    agg = defaultdict(list)
    for n, s, e, _, _ in rows:
        agg[short(n)].append((e - s) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'kernel':48s} {'calls':>7s} {'avg us':>9s} {'min us':>9s} {'total %':>8s}")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n:48s} {len(v):7d} {sum(v) / len(v):9.2f} {min(v):9.2f} {100 * sum(v) / tot:8.1f}")
    if a.timeline:
        prev = None
        for n, s, e, st, _ in rows[-a.timeline:]:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"  stream {st}  gap {gap:8.2f} us  dur {(e - s) / 1e3:8.2f} us  {short(n)}")
            prev = e
    return 0


if __name__ == "__main__":
    sys.exit(main())

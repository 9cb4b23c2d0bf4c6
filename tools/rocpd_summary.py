#!/usr/bin/env python3
"""Per-kernel summary and dispatch timeline gaps from a rocprofv3 SQLite
result (`rocprofv3 --kernel-trace -d DIR -o run`).

    python tools/rocpd_summary.py gpurun_out/x/prof/run_results.db [--timeline N]
"""
import argparse
import sqlite3
import sys
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches with gaps")
    ap.add_argument("--skip", type=int, default=0, help="ignore the first N dispatches")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = list(c.execute(f"select {name_col}, start, end, stream_id from kernels order by start"))[a.skip:]
    agg = defaultdict(list)
    for n, s, e, _ in rows:
        agg[n.split("(")[0][:70]].append((e - s) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'kernel':70s} {'calls':>7s} {'avg us':>9s} {'min us':>9s} {'total %':>8s}")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n:70s} {len(v):7d} {sum(v) / len(v):9.2f} {min(v):9.2f} {100 * sum(v) / tot:8.1f}")
    if a.timeline:
        prev = None
        for n, s, e, st in rows[-a.timeline:]:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"  stream {st}  gap {gap:8.2f} us  dur {(e - s) / 1e3:8.2f} us  {n.split('(')[0][:60]}")
            prev = e
    return 0


if __name__ == "__main__":
    sys.exit(main())

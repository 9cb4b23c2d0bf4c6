#!/usr/bin/env python3
"""Summarise a rocprofv3 (ROCm 7.2) SQLite output: per-kernel dispatch count,
total / mean / min / max device time, share of the total, VGPR/SGPR/LDS.
Also reads `--pmc` counter tables when present.

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--md]
"""

import argparse
import sqlite3
import sys
from collections import defaultdict


def table(cur, prefix):
    rows = cur.execute("select name from sqlite_master where type='table' and name like ?", (prefix + "%",)).fetchall()
    return rows[0][0] if rows else None


def summarise(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    kd = table(cur, "rocpd_kernel_dispatch")
    ks = table(cur, "rocpd_info_kernel_symbol")
    sym = {}
    for kid, name, disp, vg, ag, sg, lds in cur.execute(
        f"select id, kernel_name, display_name, arch_vgpr_count, accum_vgpr_count, sgpr_count, group_segment_size from {ks}"
    ):
        sym[kid] = (disp or name, vg, ag, sg, lds)
    agg = defaultdict(list)
    for kid, start, end in cur.execute(f"select kernel_id, start, end from {kd}"):
        agg[kid].append((end - start) * 1e-3)  # ns → µs
    out = []
    total = sum(sum(v) for v in agg.values()) or 1.0
    for kid, ts in agg.items():
        name, vg, ag, sg, lds = sym.get(kid, (str(kid), 0, 0, 0, 0))
        out.append(dict(kernel=name, calls=len(ts), total_us=sum(ts), mean_us=sum(ts) / len(ts), min_us=min(ts),
                        max_us=max(ts), pct=100.0 * sum(ts) / total, vgpr=vg, agpr=ag, sgpr=sg, lds=lds))
    out.sort(key=lambda r: -r["total_us"])
    pmc = []
    pe = table(cur, "rocpd_pmc_event")
    ip = table(cur, "rocpd_info_pmc")
    if pe and ip:
        try:
            names = {i: n for i, n in cur.execute(f"select id, name from {ip}")}
            acc = defaultdict(float)
            for pid, val in cur.execute(f"select pmc_id, value from {pe}"):
                acc[names.get(pid, pid)] += val
            pmc = sorted(acc.items())
        except sqlite3.Error:
            pass
    return out, pmc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--md", action="store_true")
    a = ap.parse_args()
    rows, pmc = summarise(a.db)
    if a.md:
        print("| kernel | calls | total µs | mean µs | min µs | max µs | % | VGPR | SGPR | LDS B |")
        print("|---|---|---|---|---|---|---|---|---|---|")
        for r in rows:
            k = r["kernel"][:90]
            print(f"| `{k}` | {r['calls']} | {r['total_us']:.1f} | {r['mean_us']:.2f} | {r['min_us']:.2f} | "
                  f"{r['max_us']:.2f} | {r['pct']:.1f} | {r['vgpr']} | {r['sgpr']} | {r['lds']} |")
    else:
        for r in rows:
            print(f"{r['pct']:5.1f}%  calls={r['calls']:6d}  mean={r['mean_us']:9.2f}us  min={r['min_us']:9.2f}  "
                  f"max={r['max_us']:9.2f}  vgpr={r['vgpr']} sgpr={r['sgpr']} lds={r['lds']}  {r['kernel'][:100]}")
    for n, v in pmc:
        print(f"PMC {n} = {v:.6g}")


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Per-dispatch PMC values of one kernel from a rocprofv3 SQLite output,
grouped into consecutive windows of `--group` dispatches (e.g. one window per
solver instance):  python tools/pmc_by_dispatch.py run_results.db --kernel kS --group 30
--by-name: one window per distinct kernel name (template instance), all its
dispatches but the first --skip."""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--kernel", default="kS")
    ap.add_argument("--group", type=int, default=1)
    ap.add_argument("--by-name", action="store_true")
    ap.add_argument("--skip", type=int, default=20)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select dispatch_id, name, duration, counter_name, counter_value from pmc_events").fetchall()
    disp = defaultdict(dict)
    for did, name, dur, cn, cv in rows:
        if a.kernel not in (name or ""):
            continue
        d = disp[did]
        d["dur"] = dur
        d["name"] = name
        d[cn] = d.get(cn, 0.0) + cv
    ids = sorted(disp)
    names = sorted({k for d in disp.values() for k in d if k not in ("dur", "name")})
    if a.by_name:
        print("n  mean_us  " + "  ".join(names) + "  kernel")
        for kn in sorted({disp[i]["name"] for i in ids}):
            body = [disp[i] for i in ids if disp[i]["name"] == kn][a.skip:]
            if not body:
                continue
            mean = sum(d["dur"] for d in body) / len(body) * 1e-3
            vals = [sum(d.get(n, 0.0) for d in body) / len(body) for n in names]
            short = kn.replace("(anonymous namespace)::", "").replace("pe::dev::", "").split("(KParams")[0]
            print(f"{len(body):4d} {mean:8.1f}  " + "  ".join(f"{v:.4g}" for v in vals) + f"  {short}")
        return
    print("window  n  mean_us  " + "  ".join(names))
    for w in range(0, len(ids), a.group):
        sel = [disp[i] for i in ids[w:w + a.group]]
        # skip the first dispatch of each window (S_0 / warm-up)
        body = sel[1:] if len(sel) > 1 else sel
        mean = sum(d["dur"] for d in body) / len(body) * 1e-3
        vals = [sum(d.get(n, 0.0) for d in body) / len(body) for n in names]
        print(f"{w // a.group:4d} {len(body):3d} {mean:8.1f}  " + "  ".join(f"{v:.4g}" for v in vals))


if __name__ == "__main__":
    main()

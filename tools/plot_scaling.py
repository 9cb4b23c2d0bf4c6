#!/usr/bin/env python3
"""Scaling chart without a plotting library: reads bench JSON lines (one per
GPU count — the driver's SCALE_*.json, or files/lines produced by
`python bench.py --gpus N`) and writes an SVG (iterations/s vs GPUs, with the
ideal-scaling line) plus a markdown table of speed-up and efficiency.

    python tools/plot_scaling.py SCALE_r01.json -o profiles/scaling.svg

The reference's equivalent is the GPU speed-up bar chart of
Этап_4_1213.pdf p.16 (made with an external tool that is not in its repo).
"""

import argparse
import json
import sys


def load(paths):
    pts = {}
    for p in paths:
        with open(p) as f:
            text = f.read()
        try:
            obj = json.loads(text)
            objs = obj if isinstance(obj, list) else obj.get("runs", [obj]) if isinstance(obj, dict) else [obj]
        except json.JSONDecodeError:
            objs = [json.loads(line) for line in text.splitlines() if line.strip().startswith("{")]
        for o in objs:
            if isinstance(o, dict) and "n_gpus" in o and "value" in o:
                pts[int(o["n_gpus"])] = float(o["value"])
    return dict(sorted(pts.items()))


def svg(pts, title):
    W, H, L, B = 560, 360, 70, 50
    xs = list(pts)
    ymax = max(max(pts.values()), pts[xs[0]] * xs[-1] / xs[0]) * 1.1
    X = lambda n: L + (W - L - 20) * (xs.index(n) / max(1, len(xs) - 1))  # noqa: E731
    Y = lambda v: H - B - (H - B - 30) * v / ymax  # noqa: E731
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{W}" height="{H}" font-family="sans-serif" font-size="12">',
           f'<text x="{W / 2}" y="18" text-anchor="middle" font-size="14">{title}</text>',
           f'<line x1="{L}" y1="{H - B}" x2="{W - 10}" y2="{H - B}" stroke="black"/>',
           f'<line x1="{L}" y1="{H - B}" x2="{L}" y2="25" stroke="black"/>']
    for t in range(6):
        v = ymax * t / 5
        out.append(f'<text x="{L - 6}" y="{Y(v) + 4}" text-anchor="end">{v:.0f}</text>')
    for n in xs:
        out.append(f'<text x="{X(n)}" y="{H - B + 18}" text-anchor="middle">{n}</text>')
    out.append(f'<text x="{W / 2}" y="{H - 10}" text-anchor="middle">GPUs</text>')
    ideal = " ".join(f"{X(n)},{Y(pts[xs[0]] * n / xs[0])}" for n in xs)
    meas = " ".join(f"{X(n)},{Y(pts[n])}" for n in xs)
    out.append(f'<polyline points="{ideal}" fill="none" stroke="#999" stroke-dasharray="5,4"/>')
    out.append(f'<polyline points="{meas}" fill="none" stroke="#c00" stroke-width="2"/>')
    for n in xs:
        out.append(f'<circle cx="{X(n)}" cy="{Y(pts[n])}" r="4" fill="#c00"/>')
    out.append(f'<text x="{L + 8}" y="40" fill="#c00">measured (PCG it/s)</text>')
    out.append(f'<text x="{L + 8}" y="56" fill="#777">ideal linear</text>')
    out.append("</svg>")
    return "\n".join(out)


def table(pts):
    n0 = next(iter(pts))
    rows = ["| GPUs | it/s | speed-up | efficiency |", "|---|---|---|---|"]
    for n, v in pts.items():
        s = v / pts[n0]
        rows.append(f"| {n} | {v:.1f} | {s:.2f} | {100 * s * n0 / n:.0f} % |")
    return "\n".join(rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("-o", "--out", default="scaling.svg")
    ap.add_argument("--title", default="8192² Jacobi-PCG, MI355X (strong scaling)")
    a = ap.parse_args()
    pts = load(a.inputs)
    if not pts:
        print("no bench records found", file=sys.stderr)
        return 1
    with open(a.out, "w") as f:
        f.write(svg(pts, a.title))
    print(table(pts))
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Per-step kernel census of a rocprofv3 SQLite trace: steps are delimited by a kernel that
runs exactly once per training step (default: the RPN NMS keep pass); the last N intervals
are averaged, so one-time work (MIOpen search, capture, warm-up) is excluded.
    python scripts/step_census.py DB [--marker nms_keep] [--last 10] [--top 80]
        [--detail REGEX]   (every call of the matching kernels in the last step, in order)"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="nms_keep")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--top", type=int, default=80)
    ap.add_argument("--sort", choices=("count", "time"), default="time")
    ap.add_argument("--detail", default="")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("PRAGMA table_info(kernels)")]
    nc = "kernel_name" if "kernel_name" in cols else "name"
    rows = con.execute(f"select {nc}, start, end from kernels order by start").fetchall()
    marks = [s for n, s, _ in rows if a.marker in n]
    if len(marks) < a.last + 1:
        raise SystemExit(f"only {len(marks)} marker kernels")
    t0, t1 = marks[-a.last - 1], marks[-1]
    agg = defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        if t0 <= s < t1:
            k = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
            agg[k][0] += 1
            agg[k][1] += (e - s) / 1000.0
    steps = a.last
    n_tot = sum(v[0] for v in agg.values()) / steps
    busy = sum(v[1] for v in agg.values()) / steps
    print(f"== {a.db}: {n_tot:.0f} kernels/step, GPU busy {busy:.0f} us/step, "
          f"wall {(t1 - t0) / 1000 / steps:.0f} us/step (last {steps} steps)")
    key = (lambda kv: -kv[1][0]) if a.sort == "count" else (lambda kv: -kv[1][1])
    for k, (c, t) in sorted(agg.items(), key=key)[:a.top]:
        print(f"{c / steps:7.1f}x {t / steps:9.1f} us {100 * t / steps / busy:5.1f}%  {k}")
    if a.detail:
        import re
        pat = re.compile(a.detail)
        gcol = [c for c in cols if "grid" in c.lower()]
        sel = ", ".join([nc, "start", "end"] + gcol)
        t0 = marks[-2]
        print(f"\n== calls matching {a.detail!r} in the last step (us, {', '.join(gcol)})")
        rows = list(con.execute(f"select {sel} from kernels where start >= ? and start < ? order by start", (t0, t1)))
        short = lambda n: n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
        for idx, r in enumerate(rows):
            if pat.search(r[0]):
                ctx = " <- ".join(short(rows[j][0])[:28] for j in range(idx - 1, max(idx - 3, -1), -1))
                nxt = short(rows[idx + 1][0])[:28] if idx + 1 < len(rows) else ""
                print(f"  {(r[2] - r[1]) / 1000.0:8.1f}  {short(r[0]):40s} {' '.join(str(g) for g in r[3:])}"
                      f"   [after: {ctx}] [next: {nxt}]")


if __name__ == "__main__":
    main()

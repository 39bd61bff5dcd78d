#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 SQLite output (run_results.db):
    python scripts/rocpd_stats.py gpurun_out/p/run_results.db [--csv out.csv] [--top 40] [--skip-first N]
Columns: kernel, calls, total_us, avg_us, pct."""
import argparse
import sqlite3
from collections import defaultdict


def load(db):
    con = sqlite3.connect(db)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("PRAGMA table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = cur.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match", default=None, help="only kernels whose name contains this")
    a = ap.parse_args()
    rows = load(a.db)
    agg = defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        if a.match and a.match not in n:
            continue
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1000.0
    tot = sum(v[1] for v in agg.values()) or 1.0
    out = sorted(agg.items(), key=lambda kv: -kv[1][1])
    lines = ["kernel,calls,total_us,avg_us,pct"]
    for n, (c, t) in out:
        lines.append(f"\"{n[:160]}\",{c},{t:.1f},{t / c:.2f},{100 * t / tot:.2f}")
    if a.csv:
        open(a.csv, "w").write("\n".join(lines) + "\n")
    print(f"total GPU time {tot:.1f} us over {sum(v[0] for v in agg.values())} dispatches")
    for l in lines[: a.top + 1]:
        print(l)


if __name__ == "__main__":
    main()

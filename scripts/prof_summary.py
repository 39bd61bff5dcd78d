#!/usr/bin/env python3
"""Short per-kernel summary of rocprofv3 SQLite outputs, per "step" (iterations given):
    python scripts/prof_summary.py DB STEPS [TOP]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db, steps = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    con = sqlite3.connect(db)
    agg = defaultdict(lambda: [0, 0.0])
    for n, s, e in con.execute("select name, start, end from kernels"):
        n = n.replace("void ", "").replace("(anonymous namespace)::", "")
        n = n.split("(")[0][:72]
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1000.0
    tot = sum(v[1] for v in agg.values())
    print(f"== {db}: GPU busy {tot / steps:.1f} us per step ({steps} steps)")
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {n:72s} {c // steps if c >= steps else c:5d}x {t / steps:9.1f} us/step {t / c:8.2f} avg {100 * t / tot:5.1f}%")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-(kernel, grid) PMC counter means + mean duration from rocprofv3 SQLite outputs, so
one kernel launched at several shapes is reported per shape:
    python scripts/rocpd_pmc_grid.py gpurun_out/x/run_results.db [more.db ...]"""
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def main():
    agg = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    dur = defaultdict(dict)
    for db in sys.argv[1:]:
        con = sqlite3.connect(db)
        cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
        gx = "grid_size_x" if "grid_size_x" in cols else "grid_x"
        wx = "workgroup_size_x" if "workgroup_size_x" in cols else "workgroup_x"
        q = f"select dispatch_id, name, {gx}, {wx}, end - start from kernels"
        meta = {}
        for disp, name, g, wgx, d in con.execute(q):
            key = (short(name), int(g) // max(int(wgx or 1), 1))
            meta[disp] = key
            dur[key][(db, disp)] = d
        for disp, cn, val in con.execute("select dispatch_id, counter_name, counter_value from pmc_events"):
            if disp in meta:
                agg[meta[disp]][cn][(db, disp)] += val
    for key in sorted(dur):
        d = list(dur[key].values())
        print(f"{key[0]}  grid={key[1]} wgs  dur={sum(d) / len(d) / 1000:.1f} us  (dispatches={len(d)})")
        for cn in sorted(agg[key]):
            v = list(agg[key][cn].values())
            print(f"   {cn:34s} {sum(v) / len(v):16.0f}")


if __name__ == "__main__":
    main()

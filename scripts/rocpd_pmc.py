#!/usr/bin/env python3
"""Per-kernel PMC counter means (summed over XCD/SE instances per dispatch, averaged over
dispatches) from rocprofv3 SQLite outputs:
    python scripts/rocpd_pmc.py gpurun_out/pmc_attn1/run_results.db [more.db ...]"""
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def main():
    agg = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for db in sys.argv[1:]:
        con = sqlite3.connect(db)
        names = {r[0]: r[1] for r in con.execute("select dispatch_id, name from kernels")}
        for disp, cn, val in con.execute("select dispatch_id, counter_name, counter_value from pmc_events"):
            agg[short(names.get(disp, "?"))][cn][disp] += val
    for k, d in agg.items():
        print(k)
        for cn in sorted(d):
            v = list(d[cn].values())
            print(f"   {cn:32s} {sum(v) / len(v):16.0f}  (dispatches={len(v)})")


if __name__ == "__main__":
    main()

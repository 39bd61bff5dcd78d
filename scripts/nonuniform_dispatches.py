#!/usr/bin/env python3
"""List the kernels of a rocprofv3 kernel trace (CSV) whose dispatches are non-uniform --
a grid size (in work-items) that is not a multiple of the workgroup size in some
dimension, i.e. a partial last workgroup.  OpenCL-style MIOpen kernels are launched
like that (hipExtModuleLaunchKernel takes global work sizes); a graph replay that
rebuilt their packets with a rounded-up grid would run work-items the kernel never
expected.

    python scripts/nonuniform_dispatches.py <kernel_trace.csv>
"""
import collections
import csv
import sys


def main(path):
    per = collections.OrderedDict()
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "?")
            g = [int(row.get(f"Grid_Size_{d}", 1) or 1) for d in "XYZ"]
            w = [int(row.get(f"Workgroup_Size_{d}", 1) or 1) for d in "XYZ"]
            nonu = any(gi % wi for gi, wi in zip(g, w))
            rec = per.setdefault(name, {"n": 0, "nonuniform": 0, "example": None, "scratch": set()})
            rec["n"] += 1
            if nonu:
                rec["nonuniform"] += 1
                rec["example"] = rec["example"] or (tuple(g), tuple(w))
            s = row.get("Scratch_Size") or row.get("Private_Segment_Size")
            if s not in (None, "", "0"):
                rec["scratch"].add(s)
    tot = sum(r["n"] for r in per.values())
    bad = {k: v for k, v in per.items() if v["nonuniform"]}
    scr = {k: v for k, v in per.items() if v["scratch"]}
    print(f"{tot} dispatches of {len(per)} kernels; {sum(v['nonuniform'] for v in bad.values())} non-uniform "
          f"dispatches of {len(bad)} kernels; {len(scr)} kernels with scratch")
    for k, v in bad.items():
        print(f"  NONUNIFORM {v['nonuniform']:5d}/{v['n']:<5d} grid {v['example'][0]} wg {v['example'][1]}  {k[:110]}")
    for k, v in scr.items():
        print(f"  SCRATCH    {v['n']:5d} sizes {sorted(v['scratch'])}  {k[:110]}")


if __name__ == "__main__":
    main(sys.argv[1])

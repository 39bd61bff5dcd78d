#!/usr/bin/env python3
"""From an AMD_LOG_LEVEL=3 log of scripts/graph_diag.py --capture-only: every hipMemcpyAsync
(and hipMemsetAsync) issued inside the capture window, with its kind / size and the kernels
launched just before it (who issued it).
    python scripts/capture_memcpy_census.py <stderr log>"""
import collections
import re
import sys


def main(path):
    inside = False
    recent = collections.deque(maxlen=3)
    kinds = collections.Counter()
    msz = collections.Counter()
    shown = 0
    for line in open(path, errors="replace"):
        if "capture-begin" in line:
            inside = True
            continue
        if "capture-end" in line:
            inside = False
            continue
        if not inside:
            continue
        m = re.search(r"ShaderName\s*:\s*(\S+)", line)
        if m:
            recent.append(m.group(1)[:90])
            continue
        if "hipMemcpyAsync (" in line or "hipMemcpyAsync(" in line or "hipMemsetAsync (" in line:
            k = re.search(r"(hipMemcpy\w+To\w+|hipMemcpyDefault)", line)
            kind = k.group(1) if k else ("memset" if "Memset" in line else "?")
            kinds[kind] += 1
            if kind == "memset":
                m2 = re.search(r"hipMemsetAsync \(\s*(0x[0-9a-f]+),\s*(-?\d+),\s*(\d+)", line)
                if m2:
                    ptr, val, size = int(m2.group(1), 16), int(m2.group(2)), int(m2.group(3))
                    msz[(size, ptr % 16, val)] += 1
            if kind not in ("hipMemcpyDeviceToDevice", "memset") and shown < 40:
                print(f"{line.strip()[:200]}\n    after: {list(recent)}")
                shown += 1
    print("inside the capture window:", dict(kinds))
    print("memsets by (bytes, dst % 16, value):")
    for (size, al, val), c in sorted(msz.items()):
        print(f"  {c:4d} x  {size:>12d} B  dst%16={al:2d}  value={val}")


if __name__ == "__main__":
    main(sys.argv[1])

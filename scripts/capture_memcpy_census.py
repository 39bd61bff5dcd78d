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
            if kind not in ("hipMemcpyDeviceToDevice", "memset") and shown < 40:
                print(f"{line.strip()[:200]}\n    after: {list(recent)}")
                shown += 1
    print("inside the capture window:", dict(kinds))


if __name__ == "__main__":
    main(sys.argv[1])

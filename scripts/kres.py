#!/usr/bin/env python3
"""Print VGPR/AGPR/scratch/LDS/occupancy per kernel of a .hip file (hipcc remarks)."""
import re, subprocess, sys
src = sys.argv[1]
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", "mxtrain/csrc", "-c", src,
                      "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r"remark: \s*([A-Za-z ]+?)(?: \[[^\]]*\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    name = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", k)[:60]
    print(f"{name:60s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} scratch={v.get('ScratchSize')} lds={v.get('LDS Size')} occ={v.get('Occupancy')}")

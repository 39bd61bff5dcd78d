#!/usr/bin/env python3
"""Which MIOpen kernels does the Mask R-CNN step run, and what do their code objects ask of
the dispatch?  Reads the MIOpen user kernel cache the training run just filled
(~/.cache/miopen/**/*.ukdb: sqlite, one compiled code object per kernel, zlib / raw), and
for every kernel prints its AMDGPU metadata: private (scratch) segment size, dynamic stack,
kernarg segment size and the hidden arguments it declares -- the dispatch-time properties a
pre-built (graph packet-capture) AQL packet has to get right.  Read-only; runs no kernel."""
import bz2
import glob
import json
import os
import re
import sqlite3
import subprocess
import sys
import tempfile
import zlib

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def blobs(db):
    con = sqlite3.connect(db)
    tables = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    print(f"{db}: tables {tables}")
    for tab in tables:
        cols = [r[1] for r in con.execute(f"pragma table_info({tab})")]
        n = con.execute(f"select count(*) from {tab}").fetchone()[0]
        print(f"  {tab}: {n} rows, columns {cols}")
        for row in con.execute(f"select * from {tab}"):
            rec = dict(zip(cols, row))
            for k, v in rec.items():
                if not isinstance(v, (bytes, bytearray)) or len(v) < 64:
                    continue
                blob = bytes(v)
                for dec in (bz2.decompress, lambda b: zlib.decompress(b), lambda b: zlib.decompress(b, -15), lambda b: b):
                    try:
                        out = dec(blob)
                    except (zlib.error, OSError, ValueError):
                        continue
                    off = out.find(b"\x7fELF")
                    if off >= 0:   # a plain code object, or one inside a clang offload bundle
                        yield rec.get("kernel_name") or rec.get("program") or rec.get("program_name") or "?", out[off:]
                        break
                    if dec is not None and out is blob:
                        print(f"    no code object in {rec.get('kernel_name')}: head {blob[:24]!r}")


def meta(blob):
    with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
        f.write(blob)
        path = f.name
    try:
        out = subprocess.run([READELF, "--notes", path], capture_output=True, text=True, timeout=60).stdout
    finally:
        os.unlink(path)
    ks = []
    for m in re.finditer(r"\.name:\s+(\S+)\n", out):
        blk = out[m.start():m.start() + 6000]
        nxt = blk.find(".name:", 10)
        if nxt > 0:
            blk = blk[:nxt]
        def g(key):
            r = re.search(r"\." + key + r":\s+(\S+)", blk)
            return r.group(1) if r else None
        hidden = sorted(set(re.findall(r"\.value_kind:\s+(hidden_\w+)", blk)))
        ks.append({"name": m.group(1), "scratch": g("private_segment_fixed_size"), "dyn_stack": g("uses_dynamic_stack"),
                   "kernarg": g("kernarg_segment_size"), "group_seg": g("group_segment_fixed_size"),
                   "hidden": hidden, "uniform_wg": g("uniform_work_group_size")})
    return ks


def main():
    dbs = glob.glob(os.path.expanduser("~/.cache/miopen/**/*.ukdb"), recursive=True)
    dbs += glob.glob(os.path.join(os.environ.get("MIOPEN_USER_DB_PATH", "/nonexistent"), "*.ukdb"))
    print("kernel dbs:", dbs)
    rows = []
    for db in dbs:
        for prog, blob in blobs(db):
            for k in meta(blob):
                k["program"] = prog
                rows.append(k)
    flag = [r for r in rows if (r["scratch"] not in (None, "0")) or r["dyn_stack"] == "true"]
    print(f"{len(rows)} kernels; {len(flag)} with scratch or a dynamic stack")
    for r in sorted(rows, key=lambda r: (r["scratch"] in (None, "0"), r["program"])):
        print(json.dumps(r))


if __name__ == "__main__":
    sys.exit(main())

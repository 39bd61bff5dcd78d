"""Image references in values / example files (reference: each
``containers/*/build_tools/build_and_push.sh`` seds the ``image:`` fields of its examples
after pushing, e.g. ``containers/megatron-deepspeed/build_tools/build_and_push.sh:59-63``;
SURVEY §2.1 C17).

    python -m mxtrain.tools.images list <dir|file>...
    python -m mxtrain.tools.images set <image> <dir|file>... [--match <substring>]

``set`` rewrites the value of every top-level or nested ``image:`` key in YAML files,
keeping comments and layout (line-based, like the reference's sed), optionally only where
the old value contains ``--match``.  Files whose image is templated (``{{ ... }}``) are
left alone.
"""
from __future__ import annotations

import argparse
import os
import re
from typing import Iterable, List, Optional, Tuple

_IMG = re.compile(r"^(?P<pre>\s*(?:-\s+)?image:\s*)(?P<q>['\"]?)(?P<val>[^'\"#\s]*)(?P=q)(?P<post>\s*(?:#.*)?)$")


def _yaml_files(paths: Iterable[str]) -> List[str]:
    out = []
    for p in paths:
        if os.path.isdir(p):
            for root, _, files in os.walk(p):
                out += [os.path.join(root, f) for f in sorted(files) if f.endswith((".yaml", ".yml"))]
        elif os.path.isfile(p):
            out.append(p)
    return sorted(out)


def list_images(paths: Iterable[str]) -> List[Tuple[str, int, str]]:
    res = []
    for f in _yaml_files(paths):
        with open(f) as fh:
            for i, line in enumerate(fh, 1):
                m = _IMG.match(line.rstrip("\n"))
                if m and m.group("val") and "{{" not in line:
                    res.append((f, i, m.group("val")))
    return res


def set_image(image: str, paths: Iterable[str], match: Optional[str] = None) -> List[str]:
    changed = []
    for f in _yaml_files(paths):
        with open(f) as fh:
            lines = fh.read().split("\n")
        dirty = False
        for i, line in enumerate(lines):
            m = _IMG.match(line)
            if not m or "{{" in line:
                continue
            old = m.group("val")
            if match and match not in old:
                continue
            if old == image:
                continue
            q = m.group("q")
            lines[i] = f"{m.group('pre')}{q}{image}{q}{m.group('post')}"
            dirty = True
        if dirty:
            with open(f, "w") as fh:
                fh.write("\n".join(lines))
            changed.append(f)
    return changed


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mxtrain.tools.images")
    sp = ap.add_subparsers(dest="cmd", required=True)
    q = sp.add_parser("list")
    q.add_argument("paths", nargs="+")
    q = sp.add_parser("set")
    q.add_argument("image")
    q.add_argument("paths", nargs="+")
    q.add_argument("--match", default=None)
    a = ap.parse_args(argv)
    if a.cmd == "list":
        for f, i, v in list_images(a.paths):
            print(f"{f}:{i}: {v}")
    else:
        for f in set_image(a.image, a.paths, a.match):
            print(f"updated {f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

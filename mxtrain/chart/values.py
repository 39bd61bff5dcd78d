"""Helm-compatible values handling: chart defaults <- ``-f`` files <- ``--set`` overrides.

Semantics follow Helm 3 (as exercised by the reference: `helm install ... -f values.yaml
--set k=v`, tutorials/maskrcnn-blog/README.md:37-49):
  * maps merge recursively, everything else (lists, scalars) is replaced;
  * a ``null`` in an override deletes the key;
  * ``--set a.b[0].c=v,x=y`` paths with typed scalars (int, float, bool, null), ``\\,``
    escapes, ``{a,b}`` lists; ``--set-string`` keeps strings.
"""
from __future__ import annotations

import copy
import re
from typing import Any, Dict, List

import yaml


def load_yaml(path: str) -> Dict[str, Any]:
    with open(path) as f:
        data = yaml.safe_load(f)
    return data or {}


def deep_merge(base: Any, over: Any) -> Any:
    if isinstance(base, dict) and isinstance(over, dict):
        out = dict(base)
        for k, v in over.items():
            if v is None:
                out.pop(k, None)
            elif k in out:
                out[k] = deep_merge(out[k], v)
            else:
                out[k] = copy.deepcopy(v)
        return out
    return copy.deepcopy(over)


def _typed(s: str, string: bool = False):
    if string:
        return s
    if s == "null":
        return None
    if s in ("true", "false"):
        return s == "true"
    if re.fullmatch(r"[-+]?\d+", s):
        try:
            return int(s)
        except ValueError:
            return s
    if re.fullmatch(r"[-+]?(\d+\.\d*|\.\d+)([eE][-+]?\d+)?", s):
        return float(s)
    if s.startswith("{") and s.endswith("}"):
        return [_typed(x.strip()) for x in _split(s[1:-1], ",")]
    return s


def _split(s: str, sep: str) -> List[str]:
    out, cur, esc, depth = [], "", False, 0
    for ch in s:
        if esc:
            cur += ch
            esc = False
            continue
        if ch == "\\":
            esc = True
            continue
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    out.append(cur)
    return out


_SEG = re.compile(r"([^.\[\]]+)((?:\[\d+\])*)")


def _path(key: str):
    parts = []
    for m in _SEG.finditer(key):
        parts.append(m.group(1))
        for idx in re.findall(r"\[(\d+)\]", m.group(2)):
            parts.append(int(idx))
    return parts


def set_path(values: Dict[str, Any], key: str, value: Any) -> None:
    parts = _path(key)
    cur: Any = values
    for i, p in enumerate(parts):
        last = i == len(parts) - 1
        nxt = parts[i + 1] if not last else None
        if isinstance(p, int):
            assert isinstance(cur, list), f"--set {key}: {parts[:i]} is not a list"
            while len(cur) <= p:
                cur.append(None)
            if last:
                cur[p] = value
            else:
                if not isinstance(cur[p], (dict, list)):
                    cur[p] = [] if isinstance(nxt, int) else {}
                cur = cur[p]
        else:
            if last:
                if value is None:
                    cur.pop(p, None)
                else:
                    cur[p] = value
            else:
                if not isinstance(cur.get(p), (dict, list)):
                    cur[p] = [] if isinstance(nxt, int) else {}
                cur = cur[p]


def apply_sets(values: Dict[str, Any], sets: List[str], string: bool = False) -> Dict[str, Any]:
    values = copy.deepcopy(values)
    for s in sets or []:
        for assignment in _split(s, ","):
            if not assignment:
                continue
            if "=" not in assignment:
                raise ValueError(f"--set expects key=value, got {assignment!r}")
            k, v = assignment.split("=", 1)
            set_path(values, k.strip(), _typed(v, string))
    return values


def merge_values(chart_values: Dict[str, Any], files: List[str] = (), sets: List[str] = (),
                 set_strings: List[str] = ()) -> Dict[str, Any]:
    v = copy.deepcopy(chart_values or {})
    for f in files or []:
        v = deep_merge(v, load_yaml(f))
    v = apply_sets(v, list(sets or []))
    v = apply_sets(v, list(set_strings or []), string=True)
    return v

"""Katib metrics collectors (reference config_maps.yaml:9-25: StdOut, File,
TensorFlowEvent) and metric strategies.

A collector turns a finished trial into ``{metric: [observations in order]}``; the
experiment then reduces each list with its strategy (``min`` / ``max`` / ``latest``;
Katib's defaults: the objective metric follows the objective type, additional metrics
take ``latest``).

* ``StdOut``          regex over the trial's logs (Katib's default TEXT format
                      ``name=value`` / ``name: value``; ``filter.metricsFormat`` overrides)
* ``File``            ``source.fileSystemPath`` {path, format: TEXT|JSON}: TEXT lines go
                      through the same regex; JSON is one object per line whose keys are
                      metric names (Katib's JSON format)
* ``TensorFlowEvent`` ``source.fileSystemPath.path`` directory of tfevents files (read by
                      mxtrain.obs.tensorboard, CRC-checked); the tag is the metric name,
                      observations are ordered by step
"""
from __future__ import annotations

import json
import os
import re
from typing import Dict, List, Optional

DEFAULT_FORMAT = r"(?P<name>[A-Za-z_][\w \-/()]*?)\s*[:=]\s*(?P<value>[-+]?\d+\.?\d*(?:[eE][-+]?\d+)?)"


def _norm(n: str) -> str:
    return n.strip().lower().replace(" ", "_")


def parse_text(text: str, names: List[str], fmt: Optional[str] = None) -> Dict[str, List[float]]:
    rx = re.compile(fmt or DEFAULT_FORMAT)
    want = {_norm(n): n for n in names}
    out: Dict[str, List[float]] = {}
    for line in text.splitlines():
        for m in rx.finditer(line):
            if "name" in rx.groupindex:
                key = _norm(m.group("name"))
                val = m.group("value")
            else:                                   # Katib style: two positional groups
                key, val = _norm(m.group(1)), m.group(2)
            # "step 10 loss: 4.5" reports metric "loss"; "lm loss: ..." reports "lm_loss"
            hit = key if key in want else next((w for w in want if key.endswith("_" + w)), None)
            if hit is not None:
                try:
                    out.setdefault(want[hit], []).append(float(val))
                except ValueError:
                    pass
    return out


def parse_json_lines(text: str, names: List[str]) -> Dict[str, List[float]]:
    out: Dict[str, List[float]] = {}
    for line in text.splitlines():
        line = line.strip()
        if not line.startswith("{"):
            continue
        try:
            rec = json.loads(line)
        except ValueError:
            continue
        for n in names:
            if n in rec:
                try:
                    out.setdefault(n, []).append(float(rec[n]))
                except (TypeError, ValueError):
                    pass
    return out


def parse_tfevents(logdir: str, names: List[str]) -> Dict[str, List[float]]:
    from ..obs.tensorboard import read_scalars
    sc = read_scalars(logdir) if os.path.isdir(logdir) else {}
    out: Dict[str, List[float]] = {}
    for n in names:
        pts = sc.get(n)
        if pts is None:   # tags are often namespaced ("train/loss"): match the leaf
            pts = next((v for k, v in sc.items() if k.split("/")[-1] == n), None)
        if pts:
            out[n] = [v for _, _, v in sorted(pts, key=lambda p: (p[0], p[1]))]
    return out


def _metrics_format(mc: dict) -> Optional[str]:
    fil = (mc.get("source") or {}).get("filter") or {}
    fmts = fil.get("metricsFormat") or []
    return fmts[0] if fmts else mc.get("format")


def collect(mc: Optional[dict], names: List[str], logs: str, subst=lambda s: s) -> Dict[str, List[float]]:
    """Run the experiment's metricsCollectorSpec over one finished trial."""
    mc = mc or {}
    kind = (mc.get("collector") or {}).get("kind") or mc.get("kind") or "StdOut"
    fmt = _metrics_format(mc)
    if kind == "StdOut":
        return parse_text(logs, names, fmt)
    fsp = (mc.get("source") or {}).get("fileSystemPath") or {}
    path = subst(fsp.get("path", ""))
    if kind == "File":
        if not os.path.exists(path):
            return {}
        with open(path, errors="replace") as f:
            text = f.read()
        if (fsp.get("format") or "TEXT").upper() == "JSON":
            return parse_json_lines(text, names)
        return parse_text(text, names, fmt)
    if kind == "TensorFlowEvent":
        return parse_tfevents(path, names)
    if kind == "None":
        return {}
    raise ValueError(f"metrics collector kind {kind} not supported (StdOut, File, TensorFlowEvent, None)")


def strategies(objective: dict) -> Dict[str, str]:
    """metric -> min|max|latest, with Katib's defaults."""
    minimize = objective.get("type", "minimize") == "minimize"
    out = {objective["objectiveMetricName"]: "min" if minimize else "max"}
    for n in objective.get("additionalMetricNames") or []:
        out[n] = "latest"
    for s in objective.get("metricStrategies") or []:
        out[s["name"]] = s.get("value", "latest")
    return out


def reduce(obs: Dict[str, List[float]], strat: Dict[str, str]) -> Dict[str, float]:
    out = {}
    for n, vals in obs.items():
        if not vals:
            continue
        s = strat.get(n, "latest")
        out[n] = min(vals) if s == "min" else max(vals) if s == "max" else vals[-1]
    return out

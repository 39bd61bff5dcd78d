"""`mxtrain lint` -- render a chart and check the manifests against what the single-node
controllers can run (the `helm lint` + admission checks of the reference platform)."""
from __future__ import annotations

from typing import List

from .render import load_chart, render_chart

KNOWN = {"PyTorchJob", "MPIJob", "RayJob", "Pod", "Deployment", "ConfigMap", "Secret", "Service",
         "PersistentVolumeClaim", "PersistentVolume", "StorageClass", "ServiceAccount"}


def _containers(m):
    spec = m.get("spec") or {}
    kind = m.get("kind")
    tmpls = []
    if kind == "Pod":
        tmpls.append(spec)
    elif kind == "Deployment":
        tmpls.append((spec.get("template") or {}).get("spec") or {})
    elif kind == "PyTorchJob":
        for rs in (spec.get("pytorchReplicaSpecs") or {}).values():
            tmpls.append(((rs or {}).get("template") or {}).get("spec") or {})
    elif kind == "MPIJob":
        for rs in (spec.get("mpiReplicaSpecs") or {}).values():
            tmpls.append(((rs or {}).get("template") or {}).get("spec") or {})
    elif kind == "RayJob":
        rc = spec.get("rayClusterSpec") or {}
        tmpls.append(((rc.get("headGroupSpec") or {}).get("template") or {}).get("spec") or {})
        for g in rc.get("workerGroupSpecs") or []:
            tmpls.append(((g.get("template") or {}).get("spec") or {}))
    for t in tmpls:
        for c in t.get("containers") or []:
            yield t, c


def lint_chart(path: str, values: List[str] = (), sets: List[str] = ()) -> List[str]:
    out = []
    try:
        chart = load_chart(path)
    except Exception as e:  # noqa: BLE001
        return [f"[ERROR] Chart.yaml: {e}"]
    for k in ("apiVersion", "name", "version"):
        if k not in chart.meta:
            out.append(f"[ERROR] Chart.yaml: {k} is required")
    if "icon" not in chart.meta:
        out.append("[INFO] Chart.yaml: icon is recommended")
    try:
        r = render_chart(chart, "lint-release", "default", list(values), list(sets))
    except Exception as e:  # noqa: BLE001
        return out + [f"[ERROR] templates/: {e}"]
    for m in r.manifests:
        kind = m.get("kind")
        name = (m.get("metadata") or {}).get("name")
        where = f"{kind}/{name}"
        if not m.get("apiVersion"):
            out.append(f"[ERROR] {where}: apiVersion missing")
        if not name:
            out.append(f"[ERROR] {kind}: metadata.name missing")
        if kind not in KNOWN:
            out.append(f"[WARNING] {where}: kind {kind} is not run by the single-node controllers")
        for podspec, c in _containers(m):
            if not (c.get("command") or c.get("args")) and kind not in ("RayJob", "MPIJob"):
                out.append(f"[WARNING] {where}: container {c.get('name')} has no command (image entrypoints "
                           "are not run)")
            vols = {v.get("name") for v in podspec.get("volumes") or []}
            for vm in c.get("volumeMounts") or []:
                if vm.get("name") not in vols:
                    out.append(f"[ERROR] {where}: volumeMount {vm.get('name')} has no volume")
    return out

"""Chart loading + rendering (the `helm template` / `helm install` front half).

A chart directory holds ``Chart.yaml``, ``values.yaml`` and ``templates/`` (``*.yaml``
manifests and ``_*.tpl`` helper files with ``define`` blocks), exactly like the
reference's charts/machine-learning/** (SURVEY §2.1 C01-C11, §2.2).  Rendering yields
the multi-document YAML text plus the parsed manifests the job controllers consume.
"""
from __future__ import annotations

import datetime as _dt
import glob
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

from .template import Engine, TemplateError
from .values import load_yaml, merge_values


@dataclass
class Chart:
    path: str
    meta: Dict[str, Any]
    values: Dict[str, Any]
    templates: Dict[str, str]
    helpers: Dict[str, str]

    @property
    def name(self):
        return self.meta.get("name", os.path.basename(self.path.rstrip("/")))


def load_chart(path: str) -> Chart:
    path = os.path.abspath(path)
    if not os.path.isfile(os.path.join(path, "Chart.yaml")):
        raise FileNotFoundError(f"{path}: not a chart (no Chart.yaml)")
    meta = load_yaml(os.path.join(path, "Chart.yaml"))
    vpath = os.path.join(path, "values.yaml")
    values = load_yaml(vpath) if os.path.exists(vpath) else {}
    templates, helpers = {}, {}
    for f in sorted(glob.glob(os.path.join(path, "templates", "**", "*"), recursive=True)):
        if os.path.isdir(f):
            continue
        rel = os.path.relpath(f, path)
        with open(f) as fh:
            text = fh.read()
        if os.path.basename(f).startswith("_"):
            helpers[rel] = text
        elif f.endswith((".yaml", ".yml", ".tpl", ".txt")):
            templates[rel] = text
    return Chart(path, meta, values, templates, helpers)


@dataclass
class Release:
    Name: str
    Namespace: str = "kubeflow-user-example-com"
    Service: str = "Helm"
    Revision: int = 1
    IsInstall: bool = True
    IsUpgrade: bool = False
    Time: _dt.datetime = field(default_factory=_dt.datetime.now)


@dataclass
class Rendered:
    release: Release
    chart: Chart
    values: Dict[str, Any]
    files: Dict[str, str]            # template path -> rendered text
    manifests: List[Dict[str, Any]]  # parsed YAML documents

    @property
    def text(self) -> str:
        out = []
        for name, body in self.files.items():
            if body.strip():
                out.append(f"---\n# Source: {self.chart.name}/{name}\n{body.strip()}\n")
        return "".join(out)

    def by_kind(self, kind: str) -> List[Dict[str, Any]]:
        return [m for m in self.manifests if m.get("kind") == kind]


def render_chart(chart: Chart, release_name: str, namespace: str = "kubeflow-user-example-com",
                 value_files: List[str] = (), sets: List[str] = (), set_strings: List[str] = (),
                 now: Optional[_dt.datetime] = None) -> Rendered:
    values = merge_values(chart.values, list(value_files), list(sets), list(set_strings))
    rel = Release(Name=release_name, Namespace=namespace)
    if now is not None:
        rel.Time = now
    ctx = {
        "Values": values,
        "Release": rel,
        "Chart": {"Name": chart.name, "Version": chart.meta.get("version", ""),
                  "AppVersion": chart.meta.get("appVersion", "")},
        "Capabilities": {"KubeVersion": {"Version": "v1.28.0"}},
        "Template": {"BasePath": f"{chart.name}/templates"},
    }
    eng = Engine()
    for name, text in chart.helpers.items():
        try:
            eng.parse(text)
        except TemplateError as e:
            raise TemplateError(f"{name}: {e}") from None
    files = {}
    manifests: List[Dict[str, Any]] = []
    for name, text in chart.templates.items():
        try:
            body = eng.render(text, ctx)
        except TemplateError as e:
            raise TemplateError(f"{chart.name}/{name}: {e}") from None
        files[name] = body
        for doc in yaml.safe_load_all(body):
            if isinstance(doc, dict) and doc:
                manifests.append(doc)
    return Rendered(rel, chart, values, files, manifests)

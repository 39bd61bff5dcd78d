"""Central dashboard for one MI355X node: the Kubeflow UI services of the reference
(``charts/ml-platform/*``) as one small HTTP server.

    python -m mxtrain dashboard [--port 8080] [--host 127.0.0.1]
        [--certfile c.crt --keyfile c.key] [--htpasswd f]

Replaces, per reference component:

* C49 central dashboard menu (``kubeflow-central-dashboard/templates/config_map.yaml:11-97``)
  -> ``GET /`` (HTML index, links below) and ``GET /api``;
* C20/C21/C21b job views (``kubectl get pytorchjobs/mpijobs/rayjobs``) ->
  ``GET /api/jobs[?namespace=]``, ``GET /api/jobs/<ns>/<name>`` (status + resources),
  ``GET /api/jobs/<ns>/<name>/logs[?pod=]``;
* C47 volumes web app -> ``GET /api/volumes`` (claims under the PV root, size, files),
  ``GET /api/volumes/<claim>?path=<rel>`` (directory listing, read-only);
* C44 Tensorboards (``Tensorboard.spec.logspath``, pvc://claim/path) -> ``POST|GET /api/tensorboards``
  (resources), ``GET /tensorboard/<name>`` (per-tag run overlays, debiased EMA smoothing,
  tag regex), ``GET /api/tensorboards?logdir=<dir>[&view=tags]``
  (every scalar series of the tfevents files under a log dir, see obs/tensorboard.py)
  and ``GET /tensorboard?logdir=<dir>`` (inline SVG charts);
* C45 Katib UI -> ``GET /api/experiments`` (HPO experiments, trials, best);
* C46 KFP UI + API server -> ``GET /api/pipelines`` (recorded pipeline runs),
  ``GET|POST /api/pipelines/defs`` (stored pipelines), ``GET|POST /api/runs``,
  ``GET /api/runs/<run>``, ``POST /api/runs/<run>/terminate`` (asynchronous runs; with
  ``cache: true`` steps whose inputs succeeded before are served from the step cache),
  ``GET|POST /api/recurringruns``, ``POST /api/recurringruns/<name>/enable|disable``
  (cron / interval schedules fired by the scheduler thread), ``GET /api/runs/<run>/lineage``,
  ``GET /api/artifacts/<id>/lineage`` (run metadata: MLMD executions / artifacts / events,
  mxtrain/mlmd.py);
* C48 profiles / KFAM -> ``GET /api/profiles``;
* C22-C26 node view (Karpenter / device plugins) -> ``GET /api/node`` (GPUs, ledger,
  node profile, sysfs power/clock samples);
* C39/C40 Istio ingress + Dex/oauth2-proxy -> optional TLS and HTTP basic auth in front of
  every route (same htpasswd format as the testing charts' nginx).

Read-only by design: jobs are created with ``mxtrain install`` / the pipeline runner.
"""
from __future__ import annotations

import argparse
import glob
import html
import json
import os
import ssl
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional

from ..runtime.storage import mxtrain_home, pv_root

MENU = [
    ("Jobs", "/api/jobs"), ("Volumes", "/api/volumes"), ("Tensorboards", "/tensorboard"),
    ("Experiments (AutoML)", "/api/experiments"), ("Pipelines", "/api/pipelines"),
    ("Profiles", "/api/profiles"), ("Node", "/api/node"),
]


# ----------------------------------------------------------------------------- data views
def jobs(namespace: Optional[str] = None) -> List[dict]:
    from ..launch import release as rel
    out = []
    for st in rel.list_releases(namespace):
        out.append({"name": st.get("name"), "namespace": st.get("namespace"), "chart": st.get("chart"),
                    "phase": st.get("phase"), "installed": st.get("installed"),
                    "kinds": sorted({r.get("kind") for r in (st.get("resources") or {}).values()
                                     if r.get("kind")})})
    return out


def job(namespace: str, name: str) -> dict:
    from ..launch import release as rel
    return rel.read_status(name, namespace)


def job_logs(namespace: str, name: str, pod: Optional[str] = None) -> str:
    from ..launch import release as rel
    if pod is not None:
        rel.check_name(pod, "pod")
    return rel.logs(name, namespace, pod)


def _du(path: str, limit: int = 200000) -> Dict:
    size = files = 0
    for root, _, fs in os.walk(path):
        for f in fs:
            try:
                size += os.path.getsize(os.path.join(root, f))
            except OSError:
                pass
            files += 1
            if files >= limit:
                return {"bytes": size, "files": files, "truncated": True}
    return {"bytes": size, "files": files}


def volumes() -> List[dict]:
    root = pv_root()
    if not os.path.isdir(root):
        return []
    out = []
    for claim in sorted(os.listdir(root)):
        d = os.path.join(root, claim)
        if os.path.isdir(d):
            out.append(dict(name=claim, path=d, reclaimPolicy="Retain", accessModes=["ReadWriteMany"],
                            **_du(d)))
    return out


def volume_browse(claim: str, rel_path: str = "") -> dict:
    from ..launch.release import check_name
    base = os.path.realpath(pv_root())
    check_name(claim, "claim")
    if claim not in os.listdir(base):
        raise FileNotFoundError(f"no volume {claim!r}")
    root = os.path.realpath(os.path.join(base, claim))
    if os.path.commonpath([base, root]) != base:
        raise PermissionError("volume escapes the PV root")
    target = os.path.realpath(os.path.join(root, rel_path.lstrip("/")))
    if not (target == root or target.startswith(root + os.sep)):
        raise PermissionError("path escapes the volume")
    if os.path.isfile(target):
        return {"claim": claim, "path": rel_path, "file": True, "bytes": os.path.getsize(target)}
    ents = []
    for e in sorted(os.listdir(target))[:1000]:
        p = os.path.join(target, e)
        ents.append({"name": e, "dir": os.path.isdir(p),
                     "bytes": os.path.getsize(p) if os.path.isfile(p) else None})
    return {"claim": claim, "path": rel_path, "entries": ents}


def tensorboard(logdir: str) -> dict:
    from ..obs.tensorboard import read_scalars
    if not os.path.isdir(logdir):
        raise FileNotFoundError(logdir)
    return {k: [{"step": s, "wall_time": w, "value": v} for s, w, v in series]
            for k, series in read_scalars(logdir).items()}


def experiments() -> List[dict]:
    out = []
    for p in sorted(glob.glob(os.path.join(mxtrain_home(), "hpo", "*", "experiment.json"))):
        with open(p) as f:
            e = json.load(f)
        out.append({"name": e.get("name"), "condition": e.get("condition"), "objective": e.get("objective"),
                    "trials": len(e.get("trials") or []), "best": e.get("best")})
    return out


def pipelines() -> List[dict]:
    from ..pipeline import runs_dir
    out = []
    for p in sorted(glob.glob(os.path.join(runs_dir(), "*.json"))):
        with open(p) as f:
            out.append(json.load(f))
    return out


def profiles() -> List[dict]:
    from .profiles import list_profiles
    return list_profiles()


def node() -> dict:
    from ..runtime.topology import NODE_PROFILES, num_gpus
    led_p = os.path.join(mxtrain_home(), "gpu-ledger.json")
    led = {}
    if os.path.exists(led_p):
        try:
            with open(led_p) as f:
                led = json.load(f)
        except ValueError:
            led = {}
    n = num_gpus()
    try:
        from ..obs.metrics import gpu_sample
        sample = gpu_sample()
    except Exception:
        sample = {}
    return {"gpus": n, "profile": f"mi355x.{n}x", "allocated": led, "free": n - len(led),
            "pv_root": pv_root(), "sysfs": sample, "known_instance_types": NODE_PROFILES}


# ----------------------------------------------------------------------------- HTML
def _svg_series(points: List[dict], w: int = 480, h: int = 160) -> str:
    if not points:
        return ""
    xs = [p["step"] for p in points]
    ys = [p["value"] for p in points]
    x0, x1 = min(xs), max(xs) or 1
    y0, y1 = min(ys), max(ys)
    if y1 == y0:
        y1 = y0 + 1
    sx = lambda x: 40 + (w - 50) * ((x - x0) / ((x1 - x0) or 1))  # noqa: E731
    sy = lambda y: h - 20 - (h - 30) * ((y - y0) / (y1 - y0))  # noqa: E731
    path = " ".join(f"{'M' if i == 0 else 'L'}{sx(x):.1f},{sy(y):.1f}" for i, (x, y) in enumerate(zip(xs, ys)))
    return (f'<svg width="{w}" height="{h}" style="border:1px solid #ccc">'
            f'<path d="{path}" fill="none" stroke="#1f77b4" stroke-width="1.5"/>'
            f'<text x="2" y="12" font-size="10">{y1:.4g}</text><text x="2" y="{h - 22}" font-size="10">{y0:.4g}</text>'
            f'<text x="40" y="{h - 4}" font-size="10">{x0}</text><text x="{w - 40}" y="{h - 4}" font-size="10">{x1}</text>'
            "</svg>")


def _index_html() -> str:
    rows = "".join(f'<li><a href="{u}">{html.escape(n)}</a></li>' for n, u in MENU)
    js = "".join(f"<tr><td>{html.escape(str(j['namespace']))}</td><td>"
                 f"<a href=\"/api/jobs/{j['namespace']}/{j['name']}\">{html.escape(str(j['name']))}</a></td>"
                 f"<td>{html.escape(str(j['chart']))}</td><td>{html.escape(str(j['phase']))}</td></tr>"
                 for j in jobs())
    return (f"<html><head><title>mxtrain dashboard</title></head><body><h2>mxtrain (MI355X node)</h2>"
            f"<ul>{rows}</ul><h3>Jobs</h3><table border=1 cellpadding=3><tr><th>namespace</th><th>name</th>"
            f"<th>chart</th><th>phase</th></tr>{js}</table></body></html>")


_COLORS = ("#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f")


def smooth_ema(values: List[float], weight: float) -> List[float]:
    """TensorBoard's scalar smoothing: debiased exponential moving average."""
    out, last, n = [], 0.0, 0
    for v in values:
        last = last * weight + (1 - weight) * v
        n += 1
        out.append(last / (1 - weight ** n) if weight > 0 else v)
    return out


def _svg_multi(series: Dict[str, List[dict]], smoothing: float, w: int = 560, h: int = 200) -> str:
    """One tag, one line per run (raw faint, smoothed solid), shared axes, legend."""
    pts = [p for v in series.values() for p in v]
    if not pts:
        return ""
    x0, x1 = min(p["step"] for p in pts), max(p["step"] for p in pts)
    y0, y1 = min(p["value"] for p in pts), max(p["value"] for p in pts)
    if y1 == y0:
        y1 = y0 + 1
    sx = lambda x: 50 + (w - 60) * ((x - x0) / ((x1 - x0) or 1))  # noqa: E731
    sy = lambda y: h - 20 - (h - 30) * ((y - y0) / (y1 - y0))  # noqa: E731
    lines, legend = [], []
    for i, (run, v) in enumerate(sorted(series.items())):
        c = _COLORS[i % len(_COLORS)]
        xs = [p["step"] for p in v]
        raw = [p["value"] for p in v]
        for ys, op in ((raw, "0.25"), (smooth_ema(raw, smoothing), "1")):
            d = " ".join(f"{'M' if j == 0 else 'L'}{sx(x):.1f},{sy(y):.1f}" for j, (x, y) in enumerate(zip(xs, ys)))
            lines.append(f'<path d="{d}" fill="none" stroke="{c}" stroke-opacity="{op}" stroke-width="1.5"/>')
        legend.append(f'<text x="{w - 150}" y="{14 + 12 * i}" font-size="10" fill="{c}">{html.escape(run)}</text>')
    return (f'<svg width="{w}" height="{h}" style="border:1px solid #ccc">{"".join(lines)}{"".join(legend)}'
            f'<text x="2" y="12" font-size="10">{y1:.4g}</text><text x="2" y="{h - 22}" font-size="10">{y0:.4g}</text>'
            f'<text x="50" y="{h - 4}" font-size="10">{x0}</text><text x="{w - 60}" y="{h - 4}" font-size="10">{x1}</text>'
            "</svg>")


def tensorboard_view(logdir: str, tag_re: Optional[str] = None) -> Dict[str, Dict[str, List[dict]]]:
    """{tag: {run: points}} -- runs are the event files' directories under logdir."""
    import re
    rx = re.compile(tag_re) if tag_re else None
    out: Dict[str, Dict[str, List[dict]]] = {}
    from ..obs.tensorboard import event_files, read_scalars
    runs = sorted({os.path.relpath(os.path.dirname(p), logdir) for p in event_files(logdir)}, key=len, reverse=True)
    for key, pts in tensorboard(logdir).items():
        run = next((r for r in runs if r != "." and key.startswith(r + "/")), ".")
        tag = key[len(run) + 1:] if run != "." else key
        if rx and not rx.search(tag):
            continue
        out.setdefault(tag, {})[run] = pts
    return out


# Tensorboard resources (Kubeflow ``Tensorboard`` CR: metadata.name + spec.logspath, with
# pvc://<claim>/<path> resolved under the PV root) -> the viewer page /tensorboard/<name>
def tensorboards_dir() -> str:
    return os.path.join(mxtrain_home(), "tensorboards")


def resolve_logspath(logspath: str) -> str:
    if logspath.startswith("pvc://"):
        claim, _, rel = logspath[len("pvc://"):].partition("/")
        from ..launch.release import check_name
        root = os.path.realpath(os.path.join(pv_root(), check_name(claim, "claim")))
        target = os.path.realpath(os.path.join(root, rel))
        if not (target == root or target.startswith(root + os.sep)):
            raise PermissionError(logspath)
        return target
    return logspath


def safe_logdir(logdir: str) -> str:
    """A log directory the viewer may read: pvc://claim/path, or a path that resolves inside
    the PV root or the mxtrain home (job logs) -- never an arbitrary server directory."""
    if logdir.startswith("pvc://"):
        return resolve_logspath(logdir)
    target = os.path.realpath(logdir)
    for root in (pv_root(), mxtrain_home()):
        r = os.path.realpath(root)
        if target == r or target.startswith(r + os.sep):
            return target
    raise PermissionError(f"log dir outside the PV root: {logdir}")


def create_tensorboard(name: str, logspath: str, namespace: str = "kubeflow-user-example-com") -> dict:
    from ..launch.release import check_name
    check_name(name, "tensorboard name")
    check_name(namespace, "namespace")
    if not logspath.startswith("pvc://"):
        raise PermissionError("Tensorboard logspath must be pvc://<claim>/<path>")
    resolve_logspath(logspath)
    os.makedirs(tensorboards_dir(), exist_ok=True)
    rec = {"name": name, "logspath": logspath, "namespace": namespace, "url": f"/tensorboard/{name}"}
    with open(os.path.join(tensorboards_dir(), name + ".json"), "w") as f:
        json.dump(rec, f)
    return rec


def list_tensorboards() -> List[dict]:
    out = []
    for p in sorted(glob.glob(os.path.join(tensorboards_dir(), "*.json"))):
        with open(p) as f:
            out.append(json.load(f))
    return out


def _tensorboard_html(logdir: Optional[str], q: Optional[Dict[str, str]] = None) -> str:
    q = q or {}
    if not logdir:
        items = "".join(f'<li><a href="{html.escape(t["url"])}">{html.escape(t["name"])}</a> '
                        f'({html.escape(t["logspath"])})</li>' for t in list_tensorboards())
        return ("<html><body><h2>Tensorboards</h2><ul>" + items + "</ul>"
                "<form action='/tensorboard'>log dir: <input name='logdir' size=60>"
                "<input type=submit value='open'></form></body></html>")
    smoothing = min(max(float(q.get("smoothing", "0.6")), 0.0), 0.999)
    view = tensorboard_view(safe_logdir(logdir), q.get("tag"))
    parts = [f"<h3>{html.escape(tag)}</h3>{_svg_multi(runs, smoothing)}" for tag, runs in sorted(view.items())]
    form = (f"<form>smoothing <input name='smoothing' value='{smoothing}' size=5> tag regex "
            f"<input name='tag' value='{html.escape(q.get('tag', ''))}'>"
            f"<input type=hidden name='logdir' value='{html.escape(logdir)}'><input type=submit value='apply'></form>")
    return f"<html><body><h2>{html.escape(logdir)}</h2>{form}{''.join(parts) or 'no scalars'}</body></html>"


# ----------------------------------------------------------------------------- server
class Auth:
    """Basic auth (htpasswd) and, with ``oidc``, bearer / session-cookie JWTs from the
    node's identity provider (mlplatform/identity.py: the Dex + oauth2-proxy roles)."""

    def __init__(self, htpasswd: Optional[str], oidc: bool = False):
        self.users: Dict[str, str] = {}
        self.oidc = oidc
        if htpasswd and os.path.exists(htpasswd):
            with open(htpasswd) as f:
                for line in f:
                    line = line.strip()
                    if ":" in line:
                        u, h = line.split(":", 1)
                        self.users[u] = h

    @property
    def enabled(self) -> bool:
        return bool(self.users) or self.oidc

    def token_user(self, header: Optional[str], cookie: Optional[str]) -> Optional[str]:
        """Email of a valid bearer token / session cookie, else None."""
        if not self.oidc:
            return None
        from .identity import verify_token
        tok = None
        if header and header.startswith("Bearer "):
            tok = header[7:].strip()
        elif cookie:
            for part in cookie.split(";"):
                k, _, v = part.strip().partition("=")
                if k == "mxtrain_session":
                    tok = v
        if not tok:
            return None
        try:
            return verify_token(tok).get("email")
        except PermissionError:
            return None

    def user(self, header: Optional[str], cookie: Optional[str] = None) -> Optional[str]:
        """The authenticated identity (token email or basic-auth user name), None when the
        server runs without auth."""
        u = self.token_user(header, cookie)
        if u:
            return u
        if self.users and header and header.startswith("Basic "):
            import base64
            try:
                return base64.b64decode(header[6:]).decode().split(":", 1)[0]
            except Exception:  # noqa: BLE001
                return None
        return None

    def ok(self, header: Optional[str], cookie: Optional[str] = None) -> bool:
        if not self.enabled:
            return True
        if self.token_user(header, cookie):
            return True
        if not self.users:
            return False
        import base64
        import hashlib
        if not header or not header.startswith("Basic "):
            return False
        try:
            u, p = base64.b64decode(header[6:]).decode().split(":", 1)
        except Exception:  # noqa: BLE001
            return False
        h = self.users.get(u)
        if h is None:
            return False
        if h.startswith("{SHA}"):
            return h[5:] == base64.b64encode(hashlib.sha1(p.encode()).digest()).decode()
        return h == p


_API_CTYPES = ("application/json", "application/yaml", "application/x-yaml", "text/yaml")


def _body_doc(body: bytes):
    """JSON or YAML request body -> object (safe loader only)."""
    import yaml
    if not body:
        return {}
    txt = body.decode("utf-8")
    try:
        return json.loads(txt)
    except ValueError:
        return yaml.safe_load(txt)


def _authorize_configs(user: Optional[str], chart_configs) -> None:
    """KFAM: an authenticated user may only start releases in namespaces whose profile
    makes them owner / contributor (mlplatform/profiles.py ``can``)."""
    if user is None:
        return
    from .profiles import can
    for c in chart_configs or []:
        ns = str((c or {}).get("namespace", "default"))
        if not can(user, "create", ns):
            raise PermissionError(f"{user} may not create jobs in namespace {ns}")


def route_post(parts: List[str], q: Dict[str, str], body: bytes, user: Optional[str] = None):
    """Pipelines API writes (KFP backend, C46):
      POST /api/pipelines/defs            {name, chart_configs, description?}  -> 201
      POST /api/runs                      {pipeline | chart_configs, name?}    -> 201 {run}
      POST /api/runs/<name>/terminate                                          -> 200"""
    from .. import pipeline as pl
    js = "application/json"
    rest = parts[1:]
    doc = _body_doc(body)
    if rest == ["pipelines", "defs"]:
        if not isinstance(doc, dict):
            raise ValueError("body must be a mapping")
        _authorize_configs(user, doc.get("chart_configs"))
        out = pl.save_pipeline(str(doc.get("name", "")), doc.get("chart_configs"), str(doc.get("description", "")))
        return 201, js, json.dumps(out)
    if rest == ["tensorboards"]:
        if not isinstance(doc, dict):
            raise ValueError("body must be a mapping")
        ns = str(doc.get("namespace", "kubeflow-user-example-com"))
        if user is not None:
            from .profiles import can
            if not can(user, "create", ns):
                raise PermissionError(f"{user} may not create Tensorboards in namespace {ns}")
        return 201, js, json.dumps(create_tensorboard(str(doc.get("name", "")), str(doc.get("logspath", "")), ns))
    if rest == ["runs"]:
        if not isinstance(doc, dict):
            raise ValueError("body must be a mapping")
        cfgs = doc.get("chart_configs")
        if cfgs is None and doc.get("pipeline"):
            cfgs = pl.get_pipeline(str(doc["pipeline"])).get("chart_configs")
        _authorize_configs(user, cfgs)
        run = pl.submit_run(chart_configs=doc.get("chart_configs"), pipeline=doc.get("pipeline"),
                            run_name=doc.get("name"), cache=bool(doc.get("cache", False)))
        return 201, js, json.dumps({"run": run})
    if rest == ["recurringruns"]:
        if not isinstance(doc, dict):
            raise ValueError("body must be a mapping")
        cfgs = pl.get_pipeline(str(doc.get("pipeline", ""))).get("chart_configs")
        _authorize_configs(user, cfgs)
        out = pl.save_recurring_run(str(doc.get("name", "")), str(doc.get("pipeline", "")), cron=doc.get("cron"),
                                    interval=doc.get("interval"), max_concurrency=int(doc.get("max_concurrency", 1)),
                                    enabled=bool(doc.get("enabled", True)), cache=bool(doc.get("cache", False)),
                                    start_time=doc.get("start_time"), end_time=doc.get("end_time"),
                                    namespaces=sorted({str((c or {}).get("namespace", "default")) for c in cfgs or []}))
        return 201, js, json.dumps(out, default=str)
    if len(rest) == 3 and rest[0] == "recurringruns" and rest[2] in ("enable", "disable"):
        if user is not None:
            from .profiles import can
            for ns in pl.get_recurring_run(rest[1]).get("namespaces") or ["default"]:
                if not can(user, "create", ns):
                    raise PermissionError(f"{user} may not change recurring runs in namespace {ns}")
        return 200, js, json.dumps(pl.set_recurring_enabled(rest[1], rest[2] == "enable"), default=str)
    if len(rest) == 3 and rest[0] == "runs" and rest[2] == "terminate":
        if user is not None:   # KFAM: only an owner / contributor of every namespace the run touches
            from .profiles import can
            for ns in pl.run_namespaces(rest[1]):
                if not can(user, "delete", ns):
                    raise PermissionError(f"{user} may not terminate runs in namespace {ns}")
        return 200, js, json.dumps({"run": rest[1], "terminating": pl.terminate_run(rest[1])})
    return 404, js, json.dumps({"error": "not found"})


def route(path: str, q: Dict[str, str], method: str = "GET", body: bytes = b"", user: Optional[str] = None):
    """(status, content-type, body) for a request; shared by the server and the tests."""
    parts = [urllib.parse.unquote(x) for x in path.strip("/").split("/") if x]
    js = "application/json"
    try:
        if method == "POST":
            if not parts or parts[0] != "api":
                return 404, js, json.dumps({"error": "not found"})
            return route_post(parts, q, body, user)
        if not parts:
            return 200, "text/html; charset=utf-8", _index_html()
        if parts == ["tensorboard"]:
            return 200, "text/html; charset=utf-8", _tensorboard_html(q.get("logdir"), q)
        if len(parts) == 2 and parts[0] == "tensorboard":
            from ..launch.release import check_name
            with open(os.path.join(tensorboards_dir(), check_name(parts[1], "tensorboard name") + ".json")) as f:
                rec = json.load(f)
            return 200, "text/html; charset=utf-8", _tensorboard_html(resolve_logspath(rec["logspath"]), q)
        if parts[0] != "api":
            return 404, js, json.dumps({"error": "not found"})
        rest = parts[1:]
        if not rest:
            return 200, js, json.dumps({"menu": [{"name": n, "href": u} for n, u in MENU]})
        k = rest[0]
        if k == "jobs" and len(rest) == 1:
            return 200, js, json.dumps(jobs(q.get("namespace")))
        if k == "jobs" and len(rest) == 3:
            return 200, js, json.dumps(job(rest[1], rest[2]), default=str)
        if k == "jobs" and len(rest) == 4 and rest[3] == "logs":
            return 200, "text/plain; charset=utf-8", job_logs(rest[1], rest[2], q.get("pod"))
        if k == "volumes" and len(rest) == 1:
            return 200, js, json.dumps(volumes())
        if k == "volumes" and len(rest) == 2:
            return 200, js, json.dumps(volume_browse(rest[1], q.get("path", "")))
        if k == "tensorboards" and "logdir" in q:
            logdir = safe_logdir(q["logdir"])
            if q.get("view") == "tags":
                return 200, js, json.dumps(tensorboard_view(logdir, q.get("tag")))
            return 200, js, json.dumps(tensorboard(logdir))
        if k == "tensorboards":
            return 200, js, json.dumps(list_tensorboards())
        if k == "experiments":
            return 200, js, json.dumps(experiments(), default=str)
        if k == "pipelines" and len(rest) == 1:
            return 200, js, json.dumps(pipelines(), default=str)
        if k == "pipelines" and rest[1:] == ["defs"]:
            from ..pipeline import list_pipeline_defs
            return 200, js, json.dumps(list_pipeline_defs(), default=str)
        if k == "pipelines" and len(rest) == 3 and rest[1] == "defs":
            from ..pipeline import get_pipeline
            return 200, js, json.dumps(get_pipeline(rest[2]), default=str)
        if k == "runs" and len(rest) == 1:
            return 200, js, json.dumps(pipelines(), default=str)
        if k == "recurringruns" and len(rest) == 1:
            from ..pipeline import list_recurring_runs
            return 200, js, json.dumps(list_recurring_runs(), default=str)
        if k == "recurringruns" and len(rest) == 2:
            from ..pipeline import get_recurring_run, next_fire
            d = get_recurring_run(rest[1])
            d["next_fire"] = next_fire(d)
            return 200, js, json.dumps(d, default=str)
        if k == "runs" and len(rest) == 2:
            from ..pipeline import get_run
            return 200, js, json.dumps(get_run(rest[1]), default=str)
        if k == "runs" and len(rest) == 3 and rest[2] == "lineage":
            from ..mlmd import run_lineage
            return 200, js, json.dumps(run_lineage(rest[1]), default=str)
        if k == "artifacts" and len(rest) == 3 and rest[2] == "lineage":
            from ..mlmd import artifact_lineage
            return 200, js, json.dumps(artifact_lineage(int(rest[1])), default=str)
        if k == "profiles":
            return 200, js, json.dumps(profiles(), default=str)
        if k == "node":
            return 200, js, json.dumps(node(), default=str)
        return 404, js, json.dumps({"error": "not found"})
    except (FileNotFoundError, KeyError) as e:
        return 404, js, json.dumps({"error": repr(e)})
    except PermissionError as e:
        return 403, js, json.dumps({"error": repr(e)})
    except ValueError as e:
        return 400, js, json.dumps({"error": repr(e)})


def make_server(host: str, port: int, auth: Auth, certfile=None, keyfile=None) -> ThreadingHTTPServer:
    loopback = host in ("127.0.0.1", "localhost", "::1")

    class H(BaseHTTPRequestHandler):
        def log_message(self, fmt, *a):
            pass

        def _public(self, method: str, u, data: bytes = b"") -> bool:
            """OIDC endpoints served without a session (token issuance, discovery)."""
            if not auth.oidc:
                return False
            from . import identity as idp
            if method == "GET" and u.path == "/.well-known/openid-configuration":
                scheme = "https" if certfile else "http"
                base = f"{scheme}://{self.headers.get('Host', host)}"
                self._send(200, "application/json", json.dumps(idp.discovery(base)))
                return True
            if method == "POST" and u.path == "/auth/token":
                ct = self.headers.get("Content-Type", "")
                if ct.startswith("application/x-www-form-urlencoded"):
                    f = {k: v[0] for k, v in urllib.parse.parse_qs(data.decode()).items()}
                else:
                    f = _body_doc(data) or {}
                try:
                    tok = idp.password_grant(str(f.get("username", "")), str(f.get("password", "")))
                except PermissionError:
                    self._send(401, "application/json", json.dumps({"error": "invalid_grant"}))
                    return True
                b = json.dumps(tok).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Set-Cookie", f"mxtrain_session={tok['access_token']}; HttpOnly; SameSite=Strict"
                                 + ("; Secure" if certfile else ""))
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)
                return True
            if method == "GET" and u.path == "/auth/userinfo":
                user = auth.token_user(self.headers.get("Authorization"), self.headers.get("Cookie"))
                if not user:
                    self._send(401, "application/json", json.dumps({"error": "invalid_token"}))
                else:
                    from .identity import load_users
                    info = load_users().get(user, {})
                    self._send(200, "application/json", json.dumps({"sub": user, "email": user,
                                                                    "groups": info.get("groups", [])}))
                return True
            return False

        def do_GET(self):  # noqa: N802
            if self._public("GET", urllib.parse.urlparse(self.path)):
                return
            if not auth.ok(self.headers.get("Authorization"), self.headers.get("Cookie")):
                self.send_response(401)
                self.send_header("WWW-Authenticate", 'Basic realm="mxtrain"')
                self.end_headers()
                return
            u = urllib.parse.urlparse(self.path)
            q = {k: v[0] for k, v in urllib.parse.parse_qs(u.query).items()}
            code, ctype, body = route(u.path, q)
            self._send(code, ctype, body)

        def _send(self, code, ctype, body):
            b = body.encode() if isinstance(body, str) else body
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(b)))
            self.end_headers()
            self.wfile.write(b)

        def do_POST(self):  # noqa: N802
            n = int(self.headers.get("Content-Length") or 0)
            if n > (1 << 20):
                self._send(413, "application/json", json.dumps({"error": "body too large"}))
                return
            data = self.rfile.read(n) if n else b""
            u = urllib.parse.urlparse(self.path)
            if self._public("POST", u, data):
                return
            if not auth.ok(self.headers.get("Authorization"), self.headers.get("Cookie")):
                self.send_response(401)
                self.send_header("WWW-Authenticate", 'Basic realm="mxtrain"')
                self.end_headers()
                return
            # writes (starting jobs) need authenticated users, except on a loopback bind
            if not auth.enabled and not loopback:
                self._send(403, "application/json", json.dumps({"error": "writes need --htpasswd or --oidc"}))
                return
            # CSRF: a browser holding cached credentials can be made to send a cross-site
            # text/plain or form POST, but not an application/json one without a preflight
            ctype = self.headers.get("Content-Type", "").split(";")[0].strip().lower()
            if ctype not in _API_CTYPES:
                self._send(415, "application/json",
                           json.dumps({"error": "Content-Type must be application/json or YAML"}))
                return
            q = {k: v[0] for k, v in urllib.parse.parse_qs(u.query).items()}
            code, ctype, body = route(u.path, q, "POST", data,
                                      auth.user(self.headers.get("Authorization"), self.headers.get("Cookie")))
            self._send(code, ctype, body)

    srv = ThreadingHTTPServer((host, port), H)
    if certfile and keyfile:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(certfile, keyfile)
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
    return srv


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mxtrain dashboard")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--certfile")
    ap.add_argument("--keyfile")
    ap.add_argument("--htpasswd")
    ap.add_argument("--oidc", action="store_true",
                    help="accept bearer / session JWTs of the node identity provider (POST /auth/token)")
    ap.add_argument("--tls-auto", action="store_true",
                    help="serve HTTPS with a certificate issued (and renewed) by the node CA")
    ap.add_argument("--no-scheduler", action="store_true", help="do not fire recurring runs from this server")
    a = ap.parse_args(argv)
    if not a.no_scheduler:
        from ..pipeline import Scheduler
        Scheduler().start()
    if a.tls_auto and not a.certfile:
        from .identity import issue_cert
        c = issue_cert("dashboard", ["localhost", a.host] if a.host not in ("127.0.0.1", "0.0.0.0") else ["localhost"],
                       ips=["127.0.0.1"])
        a.certfile, a.keyfile = c["cert"], c["key"]
    srv = make_server(a.host, a.port, Auth(a.htpasswd, oidc=a.oidc), a.certfile, a.keyfile)
    print(f"mxtrain dashboard on {'https' if a.certfile else 'http'}://{a.host}:{srv.server_address[1]}/",
          flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

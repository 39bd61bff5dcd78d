"""Sequential chart pipeline (replaces the KFP helm-charts component + pipeline;
SURVEY §2.1 C52/C53, §3.6).

``run_pipeline(chart_configs)`` installs each chart config in order, waits for every job
resource of the release to finish and always uninstalls it; the first failure stops the
pipeline and returns "Failure".  The chart-config keys are the reference component's:

    release_name, namespace (default "default"), repo_url, path | chart (+ version, branch),
    values (dict), timeout, pod_check_secs (300), pod_error_timeout (1800),
    pod_complete_timeout (7 days)

Differences from the reference, deliberately:
* the exit code of install/wait is kept when uninstall succeeds (the reference's
  ``exit_code = uninstall() and exit_code`` masks failures, helm_charts_component.py:38);
* ``repo_url`` pointing at a remote git host resolves to this checkout (offline node);
  a local directory or file:// URL is used as is;
* polling is event-driven (status.json) instead of fixed 60 s sleeps; the *timeouts* keep
  their meaning: Pending longer than pod_error_timeout or Running longer than
  pod_complete_timeout fails the config.
"""
from __future__ import annotations

import json
import os
import signal
import sys
import tempfile
import threading
import time
from typing import Dict, List, Optional

import yaml

from .launch import release as rel
from .launch.pods import REPO_ROOT


def resolve_chart(cfg: Dict) -> str:
    repo = cfg.get("repo_url") or REPO_ROOT
    if repo.startswith("file://"):
        repo = repo[len("file://"):]
    if not os.path.isdir(repo):
        repo = REPO_ROOT        # remote git URL: the node is offline, use this checkout
    if cfg.get("path"):
        p = os.path.join(repo, cfg["path"])
        if os.path.isdir(p):
            return p
        raise FileNotFoundError(f"chart path {cfg['path']} not found under {repo}")
    chart = cfg.get("chart")
    if not chart:
        raise ValueError("chart config needs 'path' or 'chart'")
    for root, dirs, files in os.walk(os.path.join(repo, "charts")):
        if os.path.basename(root) == chart and "Chart.yaml" in files:
            return root
    raise FileNotFoundError(f"chart {chart} not found under {repo}/charts")


class ChartHandler:
    def __init__(self, cfg: Dict, log=print, cancel: Optional[threading.Event] = None):
        self.cfg = cfg
        self.log = log
        self.name = cfg["release_name"]
        self.ns = cfg.get("namespace", "default")
        self._installed = False
        self.cancel = cancel

    def __call__(self) -> int:
        # signal handlers only from the main thread (API-server runs execute in threads)
        main = threading.current_thread() is threading.main_thread()
        prev = {s: signal.signal(s, self._on_signal) for s in (signal.SIGINT, signal.SIGTERM)} if main else {}
        exit_code = 1
        try:
            exit_code = self.install()
            if exit_code == 0:
                exit_code = self.wait()
        except Exception as e:  # noqa: BLE001 -- reported, counted as failure
            self.log(f"{type(e).__name__}: {e}")
            exit_code = 1
        finally:
            un = self.uninstall()
            exit_code = exit_code or un
            for s, h in prev.items():
                signal.signal(s, h)
        return exit_code

    def _on_signal(self, signum, frame):
        self.uninstall()
        sys.exit(f"Signal: {signum}")

    def install(self) -> int:
        chart = resolve_chart(self.cfg)
        files = []
        if self.cfg.get("values"):
            f = tempfile.NamedTemporaryFile("w", prefix="values", suffix=".yaml", delete=False)
            yaml.safe_dump(self.cfg["values"], f, default_flow_style=False)
            f.close()
            files.append(f.name)
        self.log(f"Install chart: {self.name} <- {chart}")
        try:
            rel.install(chart, self.name, self.ns, files)
        except Exception as e:  # noqa: BLE001
            self.log(f"Release {self.name} failed: {e}")
            return 1
        finally:
            for f in files:
                os.unlink(f)
        self._installed = True
        self.log(f"Release {self.name} successful")
        return 0

    def wait(self) -> int:
        complete_timeout = float(self.cfg.get("pod_complete_timeout", 7 * 24 * 3600))
        error_timeout = float(self.cfg.get("pod_error_timeout", 1800))
        check = min(float(self.cfg.get("pod_check_secs", 300)), 1.0)
        t0 = time.time()
        while True:
            if self.cancel is not None and self.cancel.is_set():
                self.log(f"release {self.name}: run terminated")
                return 1
            try:
                st = rel.read_status(self.name, self.ns)
            except FileNotFoundError:
                return 0     # deleted under us == Succeeded (reference semantics)
            phase = st.get("phase")
            if phase == "Succeeded":
                return 0
            if phase in ("Failed", "Unknown", "Terminated"):
                self.log(f"release {self.name}: {phase} {st.get('message', '')}")
                return 1
            el = time.time() - t0
            if phase == "Pending" and el > error_timeout:
                return 1
            if phase == "Running" and el > complete_timeout:
                return 1
            time.sleep(check)

    def uninstall(self) -> int:
        if not self._installed:
            return 0
        self._installed = False
        try:
            rel.uninstall(self.name, self.ns, keep_history=True)
            self.log(f"Uninstall release: {self.name} successful")
            return 0
        except Exception as e:  # noqa: BLE001
            self.log(f"Uninstall release: {self.name} failed: {e}")
            return 1


def runs_dir() -> str:
    from .runtime.storage import mxtrain_home
    return os.path.join(mxtrain_home(), "pipelines", "runs")


def run_pipeline(chart_configs: List[Dict], log=print, run_name: Optional[str] = None,
                 cancel: Optional[threading.Event] = None, pipeline: Optional[str] = None) -> str:
    """Sequential install -> wait -> uninstall of every chart config; "Failure" at the first
    failing step.  The run (steps, timings, result, KFP-style status Running / Succeeded /
    Failed / Terminated) is recorded under ``$MXTRAIN_HOME/pipelines/runs/`` (KFP run
    history, C46; shown and driven by the dashboard's pipelines API)."""
    from .launch.release import check_name
    run_name = check_name(run_name or time.strftime("run-%Y%m%d-%H%M%S"), "run name")
    rec = {"name": run_name, "pipeline": pipeline, "started": time.time(), "steps": [], "result": None,
           "status": "Running"}

    def _save():
        os.makedirs(runs_dir(), exist_ok=True)
        tmp = os.path.join(runs_dir(), f".{run_name}.json.tmp")
        with open(tmp, "w") as f:
            json.dump(rec, f, indent=1, default=str)
        os.replace(tmp, os.path.join(runs_dir(), run_name + ".json"))

    _save()
    result = "Success"
    for cfg in chart_configs:
        if cancel is not None and cancel.is_set():
            result = "Failure"
            break
        t0 = time.time()
        rc = ChartHandler(cfg, log, cancel)()
        rec["steps"].append({"release": cfg.get("release_name"), "namespace": cfg.get("namespace"),
                             "chart": cfg.get("chart") or cfg.get("path"), "exit_code": rc,
                             "seconds": round(time.time() - t0, 2)})
        _save()
        if rc > 0:
            result = "Failure"
            break
    rec["result"] = result
    rec["status"] = ("Terminated" if cancel is not None and cancel.is_set()
                     else "Succeeded" if result == "Success" else "Failed")
    rec["finished"] = time.time()
    _save()
    return result


# ------------------------------------------------------------ pipelines API (KFP backend)
# Stored pipeline definitions (``pipelines/defs/<name>.yaml``: {chart_configs: [...]}) and
# asynchronous runs in server threads, with terminate -- the KFP API server's pipeline /
# run / terminate surface (reference: charts/ml-platform/kubeflow-pipelines, used by
# kfp/pipelines/helm_charts_pipeline.py) over this node's chart runner.
_RUNS: Dict[str, Dict] = {}
_RUNS_LOCK = threading.Lock()


def defs_dir() -> str:
    from .runtime.storage import mxtrain_home
    return os.path.join(mxtrain_home(), "pipelines", "defs")


def save_pipeline(name: str, chart_configs: List[Dict], description: str = "") -> Dict:
    from .launch.release import check_name
    check_name(name, "pipeline name")
    if not isinstance(chart_configs, list) or not all(isinstance(c, dict) and c.get("release_name")
                                                       for c in chart_configs):
        raise ValueError("chart_configs must be a list of chart configs with release_name")
    for c in chart_configs:
        check_name(str(c["release_name"]), "release name")
        check_name(str(c.get("namespace", "default")), "namespace")
    os.makedirs(defs_dir(), exist_ok=True)
    doc = {"name": name, "description": description, "created": time.time(), "chart_configs": chart_configs}
    with open(os.path.join(defs_dir(), name + ".yaml"), "w") as f:
        yaml.safe_dump(doc, f, default_flow_style=False)
    return {"name": name, "steps": len(chart_configs)}


def get_pipeline(name: str) -> Dict:
    from .launch.release import check_name
    with open(os.path.join(defs_dir(), check_name(name, "pipeline name") + ".yaml")) as f:
        return yaml.safe_load(f)


def list_pipeline_defs() -> List[Dict]:
    import glob
    out = []
    for p in sorted(glob.glob(os.path.join(defs_dir(), "*.yaml"))):
        with open(p) as f:
            d = yaml.safe_load(f) or {}
        out.append({"name": d.get("name"), "description": d.get("description", ""),
                    "steps": len(d.get("chart_configs") or [])})
    return out


def submit_run(chart_configs: Optional[List[Dict]] = None, pipeline: Optional[str] = None,
               run_name: Optional[str] = None, log=None) -> str:
    """Start a run (a stored pipeline or inline chart configs) in a background thread;
    returns the run name.  Status: ``get_run``; stop: ``terminate_run``."""
    from .launch.release import check_name
    if chart_configs is None:
        if not pipeline:
            raise ValueError("need a pipeline name or chart_configs")
        chart_configs = list(get_pipeline(pipeline).get("chart_configs") or [])
    run_name = check_name(run_name or f"run-{time.strftime('%Y%m%d-%H%M%S')}-{os.getpid()}-{len(_RUNS)}",
                          "run name")
    cancel = threading.Event()
    logs: List[str] = []

    def body():
        run_pipeline(chart_configs, log=(log or logs.append), run_name=run_name, cancel=cancel, pipeline=pipeline)

    t = threading.Thread(target=body, name=f"pipeline-{run_name}", daemon=True)
    with _RUNS_LOCK:
        if run_name in _RUNS:
            raise ValueError(f"run {run_name} exists")
        _RUNS[run_name] = {"thread": t, "cancel": cancel, "logs": logs,
                           "namespaces": sorted({str((c or {}).get("namespace", "default")) for c in chart_configs})}
    t.start()
    return run_name


def get_run(name: str) -> Dict:
    from .launch.release import check_name
    p = os.path.join(runs_dir(), check_name(name, "run name") + ".json")
    with _RUNS_LOCK:
        live = _RUNS.get(name)
    if not os.path.exists(p):
        if live is not None:
            return {"name": name, "status": "Pending", "steps": []}
        raise FileNotFoundError(name)
    with open(p) as f:
        rec = json.load(f)
    if live is not None:
        rec["log"] = list(live["logs"])[-50:]
    return rec


def run_namespaces(name: str) -> List[str]:
    """Namespaces a run installs releases into (the KFAM check of terminate)."""
    with _RUNS_LOCK:
        live = _RUNS.get(name)
    if live is not None:
        return list(live["namespaces"])
    try:
        return sorted({str(s.get("namespace") or "default") for s in get_run(name).get("steps", [])})
    except FileNotFoundError:
        return []


def terminate_run(name: str) -> bool:
    with _RUNS_LOCK:
        live = _RUNS.get(name)
    if live is None:
        return False
    live["cancel"].set()
    return True


def wait_run(name: str, timeout: Optional[float] = None) -> Dict:
    with _RUNS_LOCK:
        live = _RUNS.get(name)
    if live is not None:
        live["thread"].join(timeout)
    return get_run(name)


def load_pipeline(path: str) -> List[Dict]:
    with open(path) as f:
        doc = yaml.safe_load(f)
    if isinstance(doc, dict):
        doc = doc.get("chart_configs", [])
    return list(doc or [])

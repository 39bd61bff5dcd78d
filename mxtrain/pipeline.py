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


# ------------------------------------------------------------ step cache (KFP cache server)
# A step's cache key is the hash of everything that determines what it runs: the chart's
# files (templates, values.yaml, Chart.yaml), the release / namespace and the values
# override.  With caching on (per run, or per chart config ``cache: true``) a step whose key
# SUCCEEDED before -- within ``max_cache_staleness`` seconds, if given -- is not run again;
# the run records it as "cached" with the execution it reused (KFP's cache-server +
# execution cache; reference: charts/ml-platform/kubeflow-pipelines/templates/
# deployments.yaml:9, the cache-server Deployment).
def cache_dir() -> str:
    from .runtime.storage import mxtrain_home
    return os.path.join(mxtrain_home(), "pipelines", "cache")


def _chart_digest(chart_dir: str) -> str:
    import hashlib
    h = hashlib.sha256()
    for root, dirs, files in sorted(os.walk(chart_dir)):
        dirs.sort()
        for f in sorted(files):
            p = os.path.join(root, f)
            h.update(os.path.relpath(p, chart_dir).encode())
            with open(p, "rb") as fh:
                h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()


def step_cache_key(cfg: Dict) -> str:
    import hashlib
    doc = {"chart": _chart_digest(resolve_chart(cfg)), "release": cfg.get("release_name"),
           "namespace": cfg.get("namespace", "default"), "values": cfg.get("values") or {}}
    return hashlib.sha256(json.dumps(doc, sort_keys=True, default=str).encode()).hexdigest()[:32]


def cache_lookup(key: str, max_staleness: Optional[float] = None) -> Optional[Dict]:
    p = os.path.join(cache_dir(), key + ".json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        ent = json.load(f)
    if max_staleness is not None and time.time() - float(ent.get("finished", 0)) > float(max_staleness):
        return None
    return ent


def cache_store(key: str, run_name: str, cfg: Dict, seconds: float) -> None:
    os.makedirs(cache_dir(), exist_ok=True)
    ent = {"key": key, "run": run_name, "release": cfg.get("release_name"), "finished": time.time(),
           "seconds": seconds}
    tmp = os.path.join(cache_dir(), f".{key}.tmp{os.getpid()}")
    with open(tmp, "w") as f:
        json.dump(ent, f)
    os.replace(tmp, os.path.join(cache_dir(), key + ".json"))


def run_pipeline(chart_configs: List[Dict], log=print, run_name: Optional[str] = None,
                 cancel: Optional[threading.Event] = None, pipeline: Optional[str] = None,
                 cache: bool = False, recurring: Optional[str] = None) -> str:
    """Sequential install -> wait -> uninstall of every chart config; "Failure" at the first
    failing step.  The run (steps, timings, result, KFP-style status Running / Succeeded /
    Failed / Terminated, and per step its cache key and whether it was served from the step
    cache) is recorded under ``$MXTRAIN_HOME/pipelines/runs/`` (KFP run history and run
    metadata, C46; shown and driven by the dashboard's pipelines API)."""
    from .launch.release import check_name
    run_name = check_name(run_name or time.strftime("run-%Y%m%d-%H%M%S"), "run name")
    rec = {"name": run_name, "pipeline": pipeline, "started": time.time(), "steps": [], "result": None,
           "status": "Running", "cache": bool(cache), "recurring_run": recurring}

    def _save():
        os.makedirs(runs_dir(), exist_ok=True)
        tmp = os.path.join(runs_dir(), f".{run_name}.json.tmp")
        with open(tmp, "w") as f:
            json.dump(rec, f, indent=1, default=str)
        os.replace(tmp, os.path.join(runs_dir(), run_name + ".json"))

    _save()
    # run metadata / lineage (MLMD, mxtrain/mlmd.py): contexts, one execution per step,
    # input and output artifacts -- best-effort, never fails the run
    from .mlmd import RunRecorder
    md = RunRecorder(run_name, pipeline, log)
    result = "Success"
    for cfg in chart_configs:
        if cancel is not None and cancel.is_set():
            result = "Failure"
            break
        t0 = time.time()
        use_cache = bool(cfg.get("cache", cache))
        try:
            chart_dir = resolve_chart(cfg)
            key = step_cache_key(cfg)
        except (FileNotFoundError, ValueError):
            chart_dir = key = None
        step = {"release": cfg.get("release_name"), "namespace": cfg.get("namespace"),
                "chart": cfg.get("chart") or cfg.get("path"), "cache_key": key, "cached": False}
        eid = md.step_started(cfg, chart_dir, key)
        step["execution_id"] = eid
        hit = cache_lookup(key, cfg.get("max_cache_staleness")) if (use_cache and key) else None
        if hit is not None:
            log(f"Step {cfg.get('release_name')}: cached (execution of run {hit.get('run')})")
            rc = 0
            step.update(cached=True, cached_from=hit.get("run"))
        else:
            rc = ChartHandler(cfg, log, cancel)()
            if rc == 0 and key:
                cache_store(key, run_name, cfg, round(time.time() - t0, 2))
        step.update(exit_code=rc, seconds=round(time.time() - t0, 2))
        md.step_finished(eid, cfg, rc, step["seconds"], cached_from=step.get("cached_from"), cache_key=key,
                         canceled=cancel is not None and cancel.is_set())
        rec["steps"].append(step)
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
               run_name: Optional[str] = None, log=None, cache: bool = False,
               recurring: Optional[str] = None) -> str:
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
        run_pipeline(chart_configs, log=(log or logs.append), run_name=run_name, cancel=cancel, pipeline=pipeline,
                     cache=cache, recurring=recurring)

    t = threading.Thread(target=body, name=f"pipeline-{run_name}", daemon=True)
    with _RUNS_LOCK:
        if run_name in _RUNS:
            raise ValueError(f"run {run_name} exists")
        _RUNS[run_name] = {"thread": t, "cancel": cancel, "logs": logs, "recurring": recurring,
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


def run_active(name: str) -> bool:
    with _RUNS_LOCK:
        live = _RUNS.get(name)
    return live is not None and live["thread"].is_alive()


# ------------------------------------------------------------ recurring runs (scheduled workflows)
# KFP's ScheduledWorkflow controller (reference: charts/ml-platform/kubeflow-pipelines/
# templates/deployments.yaml:587, ml-pipeline-scheduledworkflow): a recurring run fires a
# stored pipeline on a cron schedule or every N seconds, never more than
# ``max_concurrency`` runs at once, optionally only between start / end times; missed
# periods are not back-filled (KFP's ``no_catchup``).  Definitions live in
# ``pipelines/recurring/<name>.yaml``; ``Scheduler.tick()`` is driven by the dashboard's
# scheduler thread (or by tests with an explicit clock).
def recurring_dir() -> str:
    from .runtime.storage import mxtrain_home
    return os.path.join(mxtrain_home(), "pipelines", "recurring")


def _cron_field(spec: str, lo: int, hi: int) -> set:
    out = set()
    for part in spec.split(","):
        step = 1
        if "/" in part:
            part, st = part.split("/", 1)
            step = int(st)
            if step <= 0:
                raise ValueError(f"cron step {st}")
        if part in ("*", "?"):
            a, b = lo, hi
        elif "-" in part:
            a, b = (int(x) for x in part.split("-", 1))
        else:
            a = b = int(part)
            if step > 1:
                b = hi
        if a < lo or b > hi or a > b:
            raise ValueError(f"cron field {spec!r} outside [{lo}, {hi}]")
        out.update(range(a, b + 1, step))
    return out


class Cron:
    """5-field (minute hour day-of-month month day-of-week) or KFP's 6-field (second
    first) cron expression; ``next_after(t)`` is the first matching second > t (local
    time).  Day-of-month / day-of-week combine as in cron: both restricted -> either."""

    def __init__(self, expr: str):
        f = expr.split()
        if len(f) == 5:
            f = ["0"] + f
        if len(f) != 6:
            raise ValueError(f"cron expression needs 5 or 6 fields: {expr!r}")
        self.expr = expr
        self.sec = _cron_field(f[0], 0, 59)
        self.min = _cron_field(f[1], 0, 59)
        self.hour = _cron_field(f[2], 0, 23)
        self.dom = _cron_field(f[3], 1, 31)
        self.mon = _cron_field(f[4], 1, 12)
        self.dow = {d % 7 for d in _cron_field(f[5], 0, 7)}    # 0 and 7 = Sunday
        self._dom_any, self._dow_any = f[3] in ("*", "?"), f[5] in ("*", "?")

    def _day_ok(self, tm) -> bool:
        dom = tm.tm_mday in self.dom
        dow = ((tm.tm_wday + 1) % 7) in self.dow     # cron: 0 = Sunday
        if self._dom_any or self._dow_any:
            return dom and dow
        return dom or dow

    def next_after(self, t: float) -> float:
        import datetime as dt
        cur = dt.datetime.fromtimestamp(int(t)) + dt.timedelta(seconds=1)
        end = cur + dt.timedelta(days=366 * 5)
        while cur < end:
            tm = cur.timetuple()
            if tm.tm_mon not in self.mon:
                cur = (cur.replace(day=1, hour=0, minute=0, second=0) + dt.timedelta(days=32)).replace(day=1)
                continue
            if not self._day_ok(tm):
                cur = cur.replace(hour=0, minute=0, second=0) + dt.timedelta(days=1)
                continue
            if tm.tm_hour not in self.hour:
                cur = cur.replace(minute=0, second=0) + dt.timedelta(hours=1)
                continue
            if tm.tm_min not in self.min:
                cur = cur.replace(second=0) + dt.timedelta(minutes=1)
                continue
            if tm.tm_sec not in self.sec:
                cur = cur + dt.timedelta(seconds=1)
                continue
            return cur.timestamp()
        raise ValueError(f"cron {self.expr!r} never fires")


def save_recurring_run(name: str, pipeline: str, cron: Optional[str] = None, interval: Optional[float] = None,
                       max_concurrency: int = 1, enabled: bool = True, cache: bool = False,
                       start_time: Optional[float] = None, end_time: Optional[float] = None,
                       namespaces: Optional[List[str]] = None) -> Dict:
    from .launch.release import check_name
    check_name(name, "recurring run name")
    get_pipeline(pipeline)   # must exist
    if (cron is None) == (interval is None):
        raise ValueError("a recurring run needs exactly one of cron / interval")
    if cron is not None:
        Cron(cron)           # validate
    if interval is not None and float(interval) <= 0:
        raise ValueError("interval must be > 0 seconds")
    if int(max_concurrency) < 1:
        raise ValueError("max_concurrency must be >= 1")
    doc = {"name": name, "pipeline": pipeline, "cron": cron, "interval": None if interval is None else float(interval),
           "max_concurrency": int(max_concurrency), "enabled": bool(enabled), "cache": bool(cache),
           "start_time": start_time, "end_time": end_time, "created": time.time(), "last_fire": None,
           "runs": [], "namespaces": namespaces or []}
    os.makedirs(recurring_dir(), exist_ok=True)
    _write_recurring(doc)
    return doc


def _write_recurring(doc: Dict) -> None:
    os.makedirs(recurring_dir(), exist_ok=True)
    tmp = os.path.join(recurring_dir(), f".{doc['name']}.tmp{os.getpid()}")
    with open(tmp, "w") as f:
        yaml.safe_dump(doc, f, default_flow_style=False)
    os.replace(tmp, os.path.join(recurring_dir(), doc["name"] + ".yaml"))


def get_recurring_run(name: str) -> Dict:
    from .launch.release import check_name
    with open(os.path.join(recurring_dir(), check_name(name, "recurring run name") + ".yaml")) as f:
        return yaml.safe_load(f)


def list_recurring_runs() -> List[Dict]:
    import glob
    out = []
    for p in sorted(glob.glob(os.path.join(recurring_dir(), "*.yaml"))):
        with open(p) as f:
            d = yaml.safe_load(f) or {}
        d["next_fire"] = next_fire(d)
        out.append(d)
    return out


def set_recurring_enabled(name: str, enabled: bool) -> Dict:
    d = get_recurring_run(name)
    d["enabled"] = bool(enabled)
    if enabled:
        d["last_fire"] = time.time()   # resume from now: no catch-up of the disabled period
    _write_recurring(d)
    return d


def next_fire(d: Dict) -> Optional[float]:
    """Next firing time of a recurring run (None: disabled or past its end time)."""
    if not d.get("enabled", True):
        return None
    base = d.get("last_fire") or max(float(d.get("start_time") or 0), float(d.get("created") or 0))
    nxt = (Cron(d["cron"]).next_after(base) if d.get("cron")
           else float(base) + float(d["interval"]))
    if d.get("start_time") and nxt < float(d["start_time"]):
        nxt = float(d["start_time"])
    if d.get("end_time") and nxt > float(d["end_time"]):
        return None
    return nxt


class Scheduler:
    """Fires due recurring runs.  ``tick(now)`` is idempotent and safe to call often."""

    def __init__(self, submit=None):
        self.submit = submit or (lambda **kw: submit_run(**kw))
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def tick(self, now: Optional[float] = None) -> List[str]:
        now = time.time() if now is None else now
        fired = []
        for d in list_recurring_runs():
            nf = d.get("next_fire")
            if nf is None or nf > now:
                continue
            active = [r for r in d.get("runs", []) if run_active(r)]
            if len(active) >= int(d.get("max_concurrency", 1)):
                # at the concurrency limit: this period is skipped (not delayed), so the
                # next fire is a full period from now, as for a fired run
                d = get_recurring_run(d["name"])
                d["last_fire"] = now
                d["skipped"] = int(d.get("skipped", 0)) + 1
                _write_recurring(d)
                continue
            run = f"{d['name']}-{time.strftime('%Y%m%d-%H%M%S', time.localtime(now))}-{len(d.get('runs', []))}"
            self.submit(pipeline=d["pipeline"], run_name=run, cache=bool(d.get("cache")), recurring=d["name"])
            d = get_recurring_run(d["name"])
            d["last_fire"] = now          # no catch-up: the next period counts from now
            d.setdefault("runs", []).append(run)
            d["runs"] = d["runs"][-100:]
            _write_recurring(d)
            fired.append(run)
        return fired

    def start(self, period: float = 5.0):
        def loop():
            while not self._stop.wait(period):
                try:
                    self.tick()
                except Exception as e:  # noqa: BLE001 -- keep the scheduler alive
                    print(f"[scheduler] {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        self._thread = threading.Thread(target=loop, name="pipeline-scheduler", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()

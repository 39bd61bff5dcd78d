"""Release store + supervisor (the `helm install` back half and the operators' reconcile
loop).

A release lives in ``$MXTRAIN_HOME/releases/<namespace>/<release>/``::

    chart.json        chart path + values files + --set list (for `status`/`upgrade`)
    values.yaml       the merged values
    manifest.yaml     the rendered multi-document YAML (what `helm get manifest` shows)
    configmaps/<cm>/  materialised ConfigMaps (train-script.sh ...)
    logs/<pod>.log    one log per replica (`mxtrain logs`)
    status.json       per-resource phase / restarts / exit codes
    supervisor.pid    the detached reconcile loop

Uninstall stops the supervisor (which stops every replica's process group) and removes
the release directory; PVC data under the PV root is retained (Retain policy).
"""
from __future__ import annotations

import json
import os
import shutil
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional

import yaml

from ..chart.render import load_chart, render_chart
from ..runtime.storage import mxtrain_home
from ..runtime.topology import NodeLedger
from .controllers import CONTROLLERS, PASSIVE_KINDS, POLL

DEFAULT_NS = "kubeflow-user-example-com"


def releases_root() -> str:
    return os.path.join(mxtrain_home(), "releases")


_NAME_RE = None


def check_name(value: str, what: str = "name") -> str:
    """Release / namespace / claim names are single path components (Kubernetes object
    names): no separators, no '..', no leading dot.  Everything that turns an API path
    segment into a file path goes through here."""
    global _NAME_RE
    if _NAME_RE is None:
        import re
        _NAME_RE = re.compile(r"^[A-Za-z0-9_][A-Za-z0-9_.\-]{0,252}$")
    if not isinstance(value, str) or not _NAME_RE.match(value) or ".." in value:
        raise PermissionError(f"invalid {what}: {value!r}")
    return value


def release_dir(name: str, namespace: str = DEFAULT_NS) -> str:
    return os.path.join(releases_root(), check_name(namespace, "namespace"), check_name(name, "release name"))


def _write_json(path: str, obj):
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump(obj, f, indent=1, default=str)
    os.replace(tmp, path)


def read_status(name: str, namespace: str = DEFAULT_NS) -> dict:
    p = os.path.join(release_dir(name, namespace), "status.json")
    if not os.path.exists(p):
        raise FileNotFoundError(f"release {namespace}/{name} not found")
    with open(p) as f:
        return json.load(f)


def list_releases(namespace: Optional[str] = None) -> List[dict]:
    out = []
    root = releases_root()
    if not os.path.isdir(root):
        return out
    for ns in sorted(os.listdir(root)):
        if namespace and ns != namespace:
            continue
        for rel in sorted(os.listdir(os.path.join(root, ns))):
            try:
                out.append(read_status(rel, ns))
            except (FileNotFoundError, ValueError):
                pass
    return out


# ---------------------------------------------------------------------------- install
def install(chart_path: str, name: str, namespace: str = DEFAULT_NS, value_files: List[str] = (),
            sets: List[str] = (), set_strings: List[str] = (), wait: bool = False,
            timeout: Optional[float] = None, launch_env: Optional[Dict[str, str]] = None) -> dict:
    """Render the chart and start (or, with ``wait``, run) the release.  ``launch_env`` is
    added to every replica's environment (profiling / debug modes, see obs/profile.py)."""
    reldir = release_dir(name, namespace)
    if os.path.exists(os.path.join(reldir, "status.json")):
        st = read_status(name, namespace)
        if st.get("phase") in ("Running", "Pending") and _supervisor_alive(reldir):
            raise RuntimeError(f"cannot re-use a name that is still in use: {namespace}/{name}")
        shutil.rmtree(reldir)
    chart = load_chart(chart_path)
    rendered = render_chart(chart, name, namespace, list(value_files), list(sets), list(set_strings))
    os.makedirs(reldir, exist_ok=True)
    with open(os.path.join(reldir, "manifest.yaml"), "w") as f:
        f.write(rendered.text)
    with open(os.path.join(reldir, "values.yaml"), "w") as f:
        yaml.safe_dump(rendered.values, f, sort_keys=False)
    if launch_env:
        _write_json(os.path.join(reldir, "launch_env.json"), dict(launch_env))
    _write_json(os.path.join(reldir, "chart.json"),
                {"chart": os.path.abspath(chart_path), "chart_name": chart.name,
                 "version": chart.meta.get("version"), "values": [os.path.abspath(v) for v in value_files],
                 "set": list(sets), "set_string": list(set_strings)})
    _write_json(os.path.join(reldir, "status.json"),
                {"name": name, "namespace": namespace, "chart": chart.name, "phase": "Pending",
                 "installed": time.strftime("%Y-%m-%dT%H:%M:%S"), "resources": {}})
    if wait:
        rc = Supervisor(reldir).run(timeout=timeout)
        st = read_status(name, namespace)
        st["exit_code"] = rc
        return st
    log = open(os.path.join(reldir, "supervisor.log"), "ab")
    p = subprocess.Popen([sys.executable, "-m", "mxtrain.launch.release", "supervise", reldir],
                         stdout=log, stderr=subprocess.STDOUT, start_new_session=True,
                         env=_supervisor_env())
    log.close()
    with open(os.path.join(reldir, "supervisor.pid"), "w") as f:
        f.write(str(p.pid))
    return read_status(name, namespace)


def _supervisor_env():
    env = dict(os.environ)
    from .pods import REPO_ROOT
    pp = env.get("PYTHONPATH", "")
    env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + pp if pp else "")
    return env


def _pid_alive(pid: int) -> bool:
    try:
        # reap it if it is our own exited child (install() without wait), else a zombie
        # would look alive
        if os.waitpid(pid, os.WNOHANG)[0] == pid:
            return False
    except ChildProcessError:
        pass
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def _supervisor_alive(reldir: str) -> bool:
    p = os.path.join(reldir, "supervisor.pid")
    if not os.path.exists(p):
        return False
    try:
        return _pid_alive(int(open(p).read().strip()))
    except ValueError:
        return False


def wait(name: str, namespace: str = DEFAULT_NS, timeout: Optional[float] = None, poll: float = 0.5) -> dict:
    t0 = time.time()
    while True:
        st = read_status(name, namespace)
        if st.get("phase") in ("Succeeded", "Failed"):
            return st
        if timeout is not None and time.time() - t0 > timeout:
            return st
        reldir = release_dir(name, namespace)
        if not _supervisor_alive(reldir) and os.path.exists(os.path.join(reldir, "supervisor.pid")):
            time.sleep(poll)
            st = read_status(name, namespace)
            if st.get("phase") not in ("Succeeded", "Failed"):
                st["phase"] = "Failed"
                st["message"] = "supervisor exited unexpectedly (see supervisor.log)"
            return st
        time.sleep(poll)


def uninstall(name: str, namespace: str = DEFAULT_NS, keep_history: bool = False) -> None:
    reldir = release_dir(name, namespace)
    if not os.path.isdir(reldir):
        raise FileNotFoundError(f"release {namespace}/{name} not found")
    pidf = os.path.join(reldir, "supervisor.pid")
    if os.path.exists(pidf):
        try:
            pid = int(open(pidf).read().strip())
            if _pid_alive(pid):
                os.killpg(pid, signal.SIGTERM)
            t0 = time.time()
            while _pid_alive(pid):
                if time.time() - t0 > 30:
                    os.killpg(pid, signal.SIGKILL)
                    break
                time.sleep(0.1)
        except (ValueError, ProcessLookupError, PermissionError):
            pass
    if keep_history:
        st = read_status(name, namespace)
        st["phase"] = "Uninstalled"
        _write_json(os.path.join(reldir, "status.json"), st)
    else:
        shutil.rmtree(reldir, ignore_errors=True)


def scale(name: str, replicas: int, namespace: str = DEFAULT_NS) -> None:
    """Ask the release's elastic PyTorchJob controller for ``replicas`` workers."""
    d = release_dir(name, namespace)
    if not os.path.isdir(d):
        raise FileNotFoundError(f"release {namespace}/{name} not found")
    if replicas < 1:
        raise ValueError("replicas must be >= 1")
    _write_json(os.path.join(d, "scale.json"), {"replicas": int(replicas), "requested": time.time()})


def logs(name: str, namespace: str = DEFAULT_NS, pod: Optional[str] = None) -> str:
    d = os.path.join(release_dir(name, namespace), "logs")
    if not os.path.isdir(d):
        return ""
    files = sorted(os.listdir(d))
    if pod:
        files = [f for f in files if f.startswith(pod)]
    out = []
    for fn in files:
        with open(os.path.join(d, fn), errors="replace") as f:
            body = f.read()
        out.append(body if pod else f"==> {fn[:-4]} <==\n{body}")
    return "\n".join(out)


# ---------------------------------------------------------------------------- supervisor
class Supervisor:
    """Reconciles every job resource of one release until all are finished."""

    def __init__(self, reldir: str):
        self.reldir = reldir
        with open(os.path.join(reldir, "manifest.yaml")) as f:
            self.manifests = [m for m in yaml.safe_load_all(f) if isinstance(m, dict) and m]
        st = json.load(open(os.path.join(reldir, "status.json")))
        self.name, self.namespace = st["name"], st["namespace"]
        self.ledger = NodeLedger(os.path.join(mxtrain_home(), "gpu-ledger.json"), f"{self.namespace}/{self.name}")
        self.controllers = []
        self.passive = []
        for m in self.manifests:
            kind = m.get("kind")
            if kind in CONTROLLERS:
                self.controllers.append(CONTROLLERS[kind](m, self.manifests, reldir, self.name, self.ledger,
                                                          status_cb=lambda c: self.write_status()))
            elif kind in PASSIVE_KINDS or kind:
                self.passive.append(f"{kind}/{(m.get('metadata') or {}).get('name')}")
        self._stopping = False
        self.phase = "Pending"
        self.message = ""

    def write_status(self):
        st = {"name": self.name, "namespace": self.namespace, "phase": self.phase, "message": self.message,
              "updated": time.strftime("%Y-%m-%dT%H:%M:%S"), "supervisor_pid": os.getpid(),
              "resources": {f"{c.kind}/{c.name}": c.status() for c in self.controllers},
              "passive": self.passive}
        try:
            prev = json.load(open(os.path.join(self.reldir, "status.json")))
            st["chart"] = prev.get("chart")
            st["installed"] = prev.get("installed")
        except (OSError, ValueError):
            pass
        _write_json(os.path.join(self.reldir, "status.json"), st)

    def _on_signal(self, signum, frame):
        self._stopping = True

    def run(self, timeout: Optional[float] = None) -> int:
        import threading
        if threading.current_thread() is not threading.main_thread():
            return self._run(timeout)   # e.g. parallel HPO trials: signals stay with the main thread
        prev = (signal.signal(signal.SIGTERM, self._on_signal), signal.signal(signal.SIGINT, self._on_signal))
        try:
            return self._run(timeout)
        finally:
            signal.signal(signal.SIGTERM, prev[0])
            signal.signal(signal.SIGINT, prev[1])

    def _run(self, timeout):
        t0 = time.time()
        try:
            for c in self.controllers:
                c.start()
        except Exception as e:  # scheduling failure (e.g. not enough GPUs) -> Failed
            self.phase, self.message = "Failed", f"{type(e).__name__}: {e}"
            for c in self.controllers:
                c.stop()
                c.release_gpus()
            self.write_status()
            return 1
        self.phase = "Running" if self.controllers else "Succeeded"
        self.write_status()
        active = list(self.controllers)
        while active and not self._stopping:
            active = [c for c in active if c.step()]
            if timeout is not None and time.time() - t0 > timeout:
                self.message = f"timeout after {timeout}s"
                break
            time.sleep(POLL)
        for c in active:
            c.stop()
            c.release_gpus()
            c.phase = "Failed" if not self._stopping else "Terminated"
        phases = [c.phase for c in self.controllers]
        if self._stopping:
            self.phase = "Terminated"
        elif any(p == "Failed" for p in phases):
            self.phase = "Failed"
            self.message = "; ".join(c.message for c in self.controllers if c.phase == "Failed" and c.message)
        else:
            self.phase = "Succeeded"
        self.write_status()
        return 0 if self.phase == "Succeeded" else 1


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) == 2 and argv[0] == "supervise":
        sys.exit(Supervisor(argv[1]).run())
    raise SystemExit("usage: python -m mxtrain.launch.release supervise <release-dir>")


if __name__ == "__main__":
    main()

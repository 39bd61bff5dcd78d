"""Replica ("pod") processes: container spec -> local process with the pod's environment,
volumes and GPU set.  Replaces kubelet + container runtime for one node.

A pod is one process group (``start_new_session``) so it can be stopped exactly -- never
by pattern.  ConfigMap/Secret volumes are materialised under the release directory,
PVCs through runtime.storage, hostPath /dev/shm is used as is.
"""
from __future__ import annotations

import json
import os
import re
import signal
import stat
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..runtime.storage import MountPlan, plan_mounts

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
WORKLOADS = os.path.join(REPO_ROOT, "mxtrain", "workloads")


@dataclass
class PodSpec:
    name: str
    command: List[str]
    env: Dict[str, str]
    workdir: str
    log_path: str
    gpus: List[int] = field(default_factory=list)
    restart_policy: str = "Never"
    role: str = ""
    index: int = 0
    cpus: List[int] = field(default_factory=list)   # NUMA-local cpuset (empty = unpinned)


class Pod:
    def __init__(self, spec: PodSpec):
        self.spec = spec
        self.proc: Optional[subprocess.Popen] = None
        self.restarts = 0
        self.returncode: Optional[int] = None
        self.started_at: Optional[float] = None
        self.finished_at: Optional[float] = None

    @property
    def phase(self) -> str:
        if self.proc is None:
            return "Pending"
        if self.returncode is None:
            return "Running"
        return "Succeeded" if self.returncode == 0 else "Failed"

    def start(self):
        os.makedirs(os.path.dirname(self.spec.log_path), exist_ok=True)
        os.makedirs(self.spec.workdir, exist_ok=True)
        log = open(self.spec.log_path, "ab", buffering=0)
        log.write(f"==== {time.strftime('%Y-%m-%dT%H:%M:%S')} start {self.spec.name} "
                  f"(restart {self.restarts}) gpus={self.spec.gpus}\n".encode())
        env = dict(self.spec.env)
        from ..runtime.affinity import preexec
        self.proc = subprocess.Popen(self.spec.command, cwd=self.spec.workdir, env=env, stdout=log,
                                     stderr=subprocess.STDOUT, start_new_session=True,
                                     preexec_fn=preexec(self.spec.cpus) if self.spec.cpus else None)
        log.close()
        self.returncode = None
        self.started_at = time.time()

    def poll(self) -> Optional[int]:
        if self.proc is not None and self.returncode is None:
            rc = self.proc.poll()
            if rc is not None:
                self.returncode = rc
                self.finished_at = time.time()
        return self.returncode

    def kill(self, grace: float = 10.0):
        """Terminate the pod's whole process group (SIGTERM, then SIGKILL)."""
        if self.proc is None or self.poll() is not None:
            return
        try:
            os.killpg(self.proc.pid, signal.SIGTERM)
        except ProcessLookupError:
            return
        t0 = time.time()
        while time.time() - t0 < grace:
            if self.poll() is not None:
                return
            time.sleep(0.1)
        try:
            os.killpg(self.proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        self.proc.wait()
        self.poll()

    def to_status(self) -> dict:
        return {"phase": self.phase, "restarts": self.restarts, "exit_code": self.returncode,
                "gpus": self.spec.gpus, "log": self.spec.log_path, "pid": self.proc.pid if self.proc else None,
                "cpus": _fmt(self.spec.cpus)}


def _fmt(cpus):
    from ..runtime.affinity import format_cpulist
    return format_cpulist(cpus) if cpus else None


# --------------------------------------------------------------------------- spec building
def materialize_configmaps(manifests: List[dict], reldir: str) -> Dict[str, str]:
    """Write every ConfigMap / Secret as files; returns name -> directory."""
    out = {}
    for m in manifests:
        kind = m.get("kind")
        if kind not in ("ConfigMap", "Secret"):
            continue
        name = m["metadata"]["name"]
        d = os.path.join(reldir, "configmaps", name)
        os.makedirs(d, exist_ok=True)
        data = dict(m.get("data") or {})
        if kind == "Secret":
            import base64
            for k, v in (m.get("data") or {}).items():
                data[k] = base64.b64decode(v).decode(errors="replace")
            data.update(m.get("stringData") or {})
        for k, v in data.items():
            p = os.path.join(d, k)
            with open(p, "w") as f:
                f.write(v if v is not None else "")
        out[name] = d
    return out


def _configmap_mounts(pod_spec: dict, cm_dirs: Dict[str, str], container: dict) -> Dict[str, str]:
    """mountPath -> materialised config dir (applying items[].mode as file mode)."""
    vols = {v.get("name"): v for v in pod_spec.get("volumes") or []}
    out = {}
    for vm in container.get("volumeMounts") or []:
        v = vols.get(vm.get("name")) or {}
        ref = v.get("configMap") or v.get("secret")
        if not ref:
            continue
        cname = ref.get("name") or ref.get("secretName")
        d = cm_dirs.get(cname)
        if d is None:
            continue
        for it in ref.get("items") or []:
            p = os.path.join(d, it.get("path", it.get("key")))
            mode = it.get("mode", ref.get("defaultMode", 0o644))
            if os.path.exists(p):
                # k8s modes are decimal in YAML (365 = 0o555); keep files at least rwx for owner
                os.chmod(p, (int(mode) | stat.S_IRWXU) & 0o777)
        out[vm["mountPath"]] = d
    return out


def container_env(container: dict) -> Dict[str, str]:
    env = {}
    for e in container.get("env") or []:
        if "value" in e:
            env[e["name"]] = "" if e["value"] is None else str(e["value"])
    return env


def base_env() -> Dict[str, str]:
    env = {k: v for k, v in os.environ.items()}
    env.setdefault("PYTHONUNBUFFERED", "1")
    # MI355X multi-process GPU sharing needs dmabuf IPC (see environment notes)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    pp = env.get("PYTHONPATH", "")
    env["PYTHONPATH"] = REPO_ROOT + (os.pathsep + pp if pp else "")
    env["MXTRAIN_WORKLOADS"] = WORKLOADS
    env["MXTRAIN_REPO"] = REPO_ROOT
    return env


def build_pod(name: str, pod_template: dict, reldir: str, cm_dirs: Dict[str, str],
              extra_env: Dict[str, str], gpus: List[int], restart_policy: str = "Never",
              container_index: int = 0, command_override: Optional[List[str]] = None,
              role: str = "", index: int = 0):
    """Return (PodSpec, MountPlan) for one replica of a pod template."""
    import copy
    pod_template = copy.deepcopy(pod_template)
    spec = pod_template.get("spec", pod_template)
    containers = spec.get("containers") or [{}]
    c = containers[container_index]
    # PodDefaults of the release's namespace (admission-webhook semantics, C50)
    from ..mlplatform.profiles import apply_pod_defaults
    ns = os.path.basename(os.path.dirname(os.path.abspath(reldir)))
    applied = apply_pod_defaults(ns, pod_template if "spec" in pod_template else {"spec": spec}, c)
    plan = plan_mounts(c.get("volumeMounts") or [], spec.get("volumes") or [],
                       extra=_configmap_mounts(spec, cm_dirs, c))
    env = base_env()
    for k, v in container_env(c).items():
        # env values may reference earlier variables with $(VAR), as in a pod spec
        env[k] = plan.rewrite(expand_k8s_vars(v, env))
    # release-wide launch options (mxtrain install --profile / --debug-mode)
    le = os.path.join(reldir, "launch_env.json")
    if os.path.exists(le):
        with open(le) as f:
            env.update({k: str(v) for k, v in json.load(f).items()})
    env.update(extra_env)
    env["HOSTNAME"] = name
    env["MXTRAIN_POD_NAME"] = name
    env["MXTRAIN_MOUNTS"] = json.dumps(plan.mounts)
    if applied:
        env["MXTRAIN_POD_DEFAULTS"] = ",".join(applied)
    if gpus:
        env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpus)
    elif "HIP_VISIBLE_DEVICES" not in os.environ:
        env.setdefault("MXTRAIN_CPU_ONLY", "1")
    cmd = list(command_override if command_override is not None else
               (list(c.get("command") or []) + list(c.get("args") or [])))
    cmd = [plan.rewrite(expand_k8s_vars(str(x), env)) for x in cmd]
    # rewrite the materialised scripts too, so hard-coded /fsx paths land on NVMe
    for mp, d in plan.mounts.items():
        if plan.mode.get(mp) == "rewrite" and d.startswith(os.path.join(reldir, "configmaps")):
            for fn in os.listdir(d):
                p = os.path.join(d, fn)
                with open(p) as f:
                    txt = f.read()
                new = plan.rewrite(txt)
                if new != txt:
                    with open(p, "w") as f:
                        f.write(new)
    if cmd and cmd[0].endswith(".sh") and os.path.isfile(cmd[0]):
        cmd = ["bash"] + cmd
    home = env.get("HOME")
    workdir = c.get("workingDir")
    workdir = plan.rewrite(expand_k8s_vars(workdir, env)) if workdir else None
    if not workdir:
        workdir = home if home and (os.path.isdir(home) or _mkdir_ok(home)) else os.path.join(reldir, "pods", name)
    log = os.path.join(reldir, "logs", f"{name}.log")
    return PodSpec(name=name, command=cmd, env=env, workdir=workdir, log_path=log, gpus=gpus,
                   restart_policy=restart_policy, role=role, index=index), plan


_K8S_VAR = re.compile(r"\$\$|\$\(([A-Za-z_][A-Za-z0-9_]*)\)")


def expand_k8s_vars(s: str, env: Dict[str, str]) -> str:
    """Kubernetes `$(VAR)` expansion in command/args against the container env; `$$`
    escapes, unknown references stay verbatim (kubelet semantics)."""
    def rep(m):
        if m.group(0) == "$$":
            return "$"
        k = m.group(1)
        return env[k] if k in env else m.group(0)
    return _K8S_VAR.sub(rep, s)


def _mkdir_ok(path: str) -> bool:
    try:
        os.makedirs(path, exist_ok=True)
        return True
    except OSError:
        return False


def python_exe() -> str:
    return sys.executable

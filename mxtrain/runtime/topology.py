"""Node topology + GPU allocation (replaces the nvidia-device-plugin / Karpenter NodePool
layer of the reference).

* GPUs are discovered from the KFD sysfs topology (no HIP call, so discovery never
  initialises the GPU in the launcher process) or from ``MXTRAIN_NUM_GPUS``.
* Resource keys ``amd.com/gpu`` (native) and ``nvidia.com/gpu`` (reference alias) both
  request MI355X GPUs; ``aws.amazon.com/neuron*`` / ``vpc.amazonaws.com/efa`` are
  accepted and ignored with a note.
* ``node_type`` / ``gpu_instance_type`` resolve through NODE_PROFILES (the reference's
  instance types keep working, mapped to their GPU count); the local node profile is
  ``mi355x.8x``.
"""
from __future__ import annotations

import glob
import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional

GPU_KEYS = ("amd.com/gpu", "nvidia.com/gpu")
IGNORED_KEYS = ("aws.amazon.com/neuron", "aws.amazon.com/neuroncore", "aws.amazon.com/neurondevice",
                "vpc.amazonaws.com/efa")

# instance type -> GPUs per node (reference instance types keep working)
NODE_PROFILES: Dict[str, int] = {
    "mi355x.8x": 8, "mi355x.4x": 4, "mi355x.2x": 2, "mi355x.1x": 1,
    "g5.xlarge": 1, "g5.2xlarge": 1, "g5.12xlarge": 4, "g5.24xlarge": 4, "g5.48xlarge": 8,
    "g4dn.xlarge": 1, "g4dn.12xlarge": 4, "p3.2xlarge": 1, "p3.8xlarge": 4, "p3.16xlarge": 8,
    "p3dn.24xlarge": 8, "p4d.24xlarge": 8, "p4de.24xlarge": 8, "p5.48xlarge": 8,
}


def _kfd_gpus() -> List[int]:
    """Indices of GPU agents in the KFD topology (nodes with a non-zero gfx target)."""
    out = []
    nodes = sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"),
                   key=lambda p: int(p.split("/")[-2]))
    for p in nodes:
        try:
            with open(p) as f:
                props = dict(line.split() for line in f if len(line.split()) == 2)
        except OSError:
            continue
        if int(props.get("gfx_target_version", "0")) != 0:
            out.append(len(out))
    return out


def num_gpus() -> int:
    env = os.environ.get("MXTRAIN_NUM_GPUS")
    if env not in (None, ""):
        return int(env)
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    n = len(_kfd_gpus())
    if vis:
        n = len([x for x in vis.split(",") if x.strip() != ""])
    return n


def gpus_requested(resources: Optional[dict]) -> int:
    """GPU count from a container `resources` block (requests, else limits)."""
    if not resources:
        return 0
    for section in ("limits", "requests"):
        sec = resources.get(section) or {}
        for k in GPU_KEYS:
            if k in sec and sec[k] not in (None, ""):
                return int(sec[k])
    return 0


def profile_gpus(node_type: Optional[str]) -> Optional[int]:
    if not node_type:
        return None
    return NODE_PROFILES.get(str(node_type))


@dataclass
class GPUAllocator:
    """Hands out disjoint GPU index sets to replicas (one rank per GPU)."""
    total: int = field(default_factory=num_gpus)
    _free: List[int] = field(default_factory=list)
    _lock: threading.Lock = field(default_factory=threading.Lock)

    def __post_init__(self):
        base = os.environ.get("HIP_VISIBLE_DEVICES")
        ids = [int(x) for x in base.split(",")] if base else list(range(self.total))
        self._free = ids[: self.total]

    def allocate(self, n: int) -> List[int]:
        with self._lock:
            if n > len(self._free):
                raise RuntimeError(f"requested {n} GPUs, only {len(self._free)} of {self.total} free "
                                   "(one MI355X per rank; reduce nnodes x nproc_per_node)")
            got, self._free = self._free[:n], self._free[n:]
            return got

    def release(self, ids: List[int]):
        with self._lock:
            self._free = sorted(set(self._free) | set(ids))


class NodeLedger(GPUAllocator):
    """GPUAllocator shared by every release on the node (the device-plugin's job): the
    owner of each GPU is recorded in ``<home>/gpu-ledger.json`` under an flock, and
    entries whose owning supervisor PID is gone are reclaimed."""

    def __init__(self, path: str, owner: str, total: Optional[int] = None):
        self.path = path
        self.owner = owner
        super().__init__(total=num_gpus() if total is None else total)

    def _locked(self, fn):
        import fcntl
        import json
        os.makedirs(os.path.dirname(self.path), exist_ok=True)
        with open(self.path + ".lock", "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                with open(self.path) as f:
                    led = json.load(f)
            except (OSError, ValueError):
                led = {}
            led = {g: o for g, o in led.items() if _pid_alive(o.get("pid", -1))}
            out = fn(led)
            tmp = self.path + ".tmp"
            with open(tmp, "w") as f:
                json.dump(led, f, indent=1)
            os.replace(tmp, self.path)
            return out

    def allocate(self, n: int) -> List[int]:
        def take(led):
            ns = self.owner.split("/", 1)[0]
            try:
                from ..mlplatform.profiles import gpu_quota
                quota = gpu_quota(ns)
            except Exception:
                quota = None
            if quota is not None:
                used = sum(1 for o in led.values() if str(o.get("owner", "")).split("/", 1)[0] == ns)
                if used + n > quota:
                    raise RuntimeError(f"exceeded quota: namespace {ns} requested {n} GPUs with "
                                       f"{used} in use, limit amd.com/gpu={quota}")
            free = [g for g in self._free if str(g) not in led]
            if n > len(free):
                busy = sorted({o["owner"] for o in led.values()})
                raise RuntimeError(f"requested {n} GPUs, only {len(free)} of {self.total} free "
                                   f"(held by {busy}); one MI355X per rank")
            got = free[:n]
            for g in got:
                led[str(g)] = {"owner": self.owner, "pid": os.getpid()}
            return got
        with self._lock:
            got = self._locked(take)
            self._free = [g for g in self._free if g not in got]
            return got

    def release(self, ids: List[int]):
        def give(led):
            for g in ids:
                led.pop(str(g), None)
        with self._lock:
            self._locked(give)
            self._free = sorted(set(self._free) | set(ids))


def _pid_alive(pid: int) -> bool:
    if pid <= 0:
        return False
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True

"""PersistentVolumeClaim -> local NVMe mapping (replaces pv-efs / pv-fsx / EFS / FSx-Lustre,
SURVEY §2.1 C27-C34, §2.4).

Every claim name maps to ``<pv_root>/<claimName>`` (``MXTRAIN_PV_ROOT``, default
``$MXTRAIN_HOME/pv``, i.e. local NVMe).  The pod-visible mount path (``/fsx``, ``/efs``)
is realised, in order of preference:

1. ``link``    -- the mount path already IS that directory, or a symlink to it can be
                  created (root in a container);
2. ``rewrite`` -- otherwise (non-root, read-only ``/``, e.g. the gpurun box) every
                  occurrence of the mount-path prefix in the replica's env values,
                  command/args and generated script is rewritten to the host directory.

Either way the directory layout *under* the mount is unchanged, so the
Megatron-DeepSpeed checkpoint tree ``/fsx/home/<rel>/checkpoints/<node_rank>/...`` keeps
its shape.  Reclaim policy is Retain: uninstall never deletes claim data.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional


def mxtrain_home() -> str:
    return os.environ.get("MXTRAIN_HOME", os.path.join(os.path.expanduser("~"), ".mxtrain"))


def pv_root() -> str:
    return os.environ.get("MXTRAIN_PV_ROOT", os.path.join(mxtrain_home(), "pv"))


@dataclass
class MountPlan:
    mounts: Dict[str, str] = field(default_factory=dict)   # mount path -> host dir
    mode: Dict[str, str] = field(default_factory=dict)     # mount path -> link|rewrite|same

    def rewrite(self, text: str) -> str:
        """Rewrite mount-path prefixes (only in 'rewrite' mode) inside a string."""
        for mp, host in sorted(self.mounts.items(), key=lambda kv: -len(kv[0])):
            if self.mode.get(mp) != "rewrite" or mp in ("/", ""):
                continue
            text = re.sub(r"(?<![\w.-])" + re.escape(mp.rstrip("/")) + r"(?=/|\b|$)", host, text)
        return text

    def rewrite_list(self, xs: List[str]) -> List[str]:
        return [self.rewrite(x) for x in xs]


def _try_link(mount_path: str, host: str) -> bool:
    try:
        if os.path.islink(mount_path):
            return os.path.realpath(mount_path) == os.path.realpath(host)
        if os.path.exists(mount_path):
            return os.path.realpath(mount_path) == os.path.realpath(host)
        parent = os.path.dirname(mount_path.rstrip("/")) or "/"
        if os.access(parent, os.W_OK):
            os.symlink(host, mount_path)
            return True
    except OSError:
        return False
    return False


def plan_mounts(volume_mounts: List[dict], volumes: List[dict], extra: Optional[Dict[str, str]] = None,
                allow_link: Optional[bool] = None) -> MountPlan:
    """Resolve a pod's volumeMounts against its volumes (PVC claims + hostPath + the
    config map, which the controller handles separately)."""
    if allow_link is None:
        allow_link = os.environ.get("MXTRAIN_PV_LINK", "1") == "1"
    by_name = {v.get("name"): v for v in volumes or []}
    plan = MountPlan()
    for vm in volume_mounts or []:
        v = by_name.get(vm.get("name"), {})
        mp = vm.get("mountPath")
        if not mp:
            continue
        if "persistentVolumeClaim" in v:
            claim = v["persistentVolumeClaim"].get("claimName")
            host = os.path.join(pv_root(), claim)
            os.makedirs(host, exist_ok=True)
            plan.mounts[mp] = host
            plan.mode[mp] = "link" if allow_link and _try_link(mp, host) else "rewrite"
        elif "hostPath" in v:
            hp = v["hostPath"].get("path")
            if v["hostPath"].get("type") == "DirectoryOrCreate" and not os.path.isdir(hp):
                try:
                    os.makedirs(hp, exist_ok=True)
                except OSError:
                    # not creatable here (read-only /, non-root): back it by local storage
                    hp = os.path.join(mxtrain_home(), "hostpath", hp.strip("/").replace("/", "_"))
                    os.makedirs(hp, exist_ok=True)
            plan.mounts[mp] = hp
            plan.mode[mp] = "same" if os.path.realpath(hp) == os.path.realpath(mp) else "rewrite"
    for mp, host in (extra or {}).items():
        plan.mounts[mp] = host
        plan.mode[mp] = "rewrite"
    return plan

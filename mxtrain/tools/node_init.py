"""Node bring-up and storage operations for one MI355X node.

The reference provisions its platform with Terraform (VPC, EKS, node groups, EFS,
FSx-for-Lustre with an S3 data-repository association, storage classes and PV/PVCs,
profiles; ``eks-cluster/terraform/aws-eks-cluster-and-nodegroup/{main,variables}.tf``,
SURVEY §2.1 C27-C42) and then stages data by hand with utility pods
(``eks-cluster/utils/{attach-pvc,stage-data}.yaml``, ``prepare-s3-bucket.sh``; C56).
On a single node the same intent is one declarative file (``infra/node.yaml``):

    python -m mxtrain node init -f infra/node.yaml      # volumes, home dirs, profiles, repo import
    python -m mxtrain node stage-data <src> pv-fsx:data/coco2017    # stage-data.yaml
    python -m mxtrain node attach-pvc                   # attach-pvc.yaml: where each claim lives
    python -m mxtrain node export pv-fsx                # FSx auto-export to the data repository

Volumes keep the reference's claim names (``pv-efs``, ``pv-fsx``) and mount paths
(``/efs``, ``/fsx``); their data lives under the PV root on local NVMe
(runtime/storage.py).  A volume's ``data_repository`` (the FSx DRA ``import_path``) is a
directory that is imported on init (auto_import) and can be exported back (auto_export),
newer-or-missing files only, like Lustre's lazy import / export policies.
"""
from __future__ import annotations

import os
import shutil
from typing import Dict, List, Optional

import yaml

from ..runtime.storage import mxtrain_home, pv_root

DEFAULT_CONFIG = {
    "cluster_name": "mi355x-node",
    "node_profile": "mi355x.8x",
    "volumes": [
        {"name": "pv-efs", "storage_class": "efs-sc", "capacity": "1000Gi",
         "access_modes": ["ReadWriteMany"], "reclaim_policy": "Retain", "mount_path": "/efs"},
        {"name": "pv-fsx", "storage_class": "fsx-sc", "capacity": "1200Gi",
         "access_modes": ["ReadWriteMany"], "reclaim_policy": "Retain", "mount_path": "/fsx",
         "mount_options": ["noatime", "flock"]},
    ],
    "home_dirs": [{"volume": "pv-efs", "path": "home"}, {"volume": "pv-fsx", "path": "home"}],
    "profiles": [{"name": "kubeflow-user-example-com", "owner": "user@example.com"}],
}


def _bytes(cap: str) -> int:
    units = {"Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30, "Ti": 1 << 40, "K": 10 ** 3, "M": 10 ** 6,
             "G": 10 ** 9, "T": 10 ** 12}
    cap = str(cap).strip()
    for u in sorted(units, key=len, reverse=True):
        if cap.endswith(u):
            return int(float(cap[: -len(u)]) * units[u])
    return int(cap)


def load_config(path: Optional[str]) -> dict:
    if not path:
        return dict(DEFAULT_CONFIG)
    with open(path) as f:
        cfg = yaml.safe_load(f) or {}
    out = dict(DEFAULT_CONFIG)
    out.update(cfg)
    return out


def sync_tree(src: str, dst: str) -> Dict[str, int]:
    """Copy files that are missing or newer (size/mtime) from src to dst."""
    copied = skipped = 0
    for root, _, files in os.walk(src):
        rel = os.path.relpath(root, src)
        droot = os.path.join(dst, rel) if rel != "." else dst
        os.makedirs(droot, exist_ok=True)
        for f in files:
            s, d = os.path.join(root, f), os.path.join(droot, f)
            try:
                ss = os.stat(s)
                if os.path.exists(d):
                    ds = os.stat(d)
                    if ds.st_size == ss.st_size and ds.st_mtime >= ss.st_mtime:
                        skipped += 1
                        continue
                shutil.copy2(s, d)
                copied += 1
            except OSError:
                continue
    return {"copied": copied, "skipped": skipped}


def init_node(cfg: dict) -> dict:
    """Create volumes, home directories, profiles and the data-repository import; the
    applied config is recorded in $MXTRAIN_HOME/node.yaml.  Idempotent."""
    from ..mlplatform import profiles as pr
    report = {"volumes": {}, "profiles": [], "warnings": []}
    root = cfg.get("pv_root") or pv_root()
    os.environ.setdefault("MXTRAIN_PV_ROOT", root)
    os.makedirs(root, exist_ok=True)
    free = shutil.disk_usage(root).free
    for v in cfg.get("volumes") or []:
        d = os.path.join(root, v["name"])
        os.makedirs(d, exist_ok=True)
        cap = _bytes(v.get("capacity", "0"))
        if cap and cap > free:
            report["warnings"].append(f"{v['name']}: capacity {v.get('capacity')} exceeds free space "
                                      f"{free / 2 ** 30:.0f} GiB on {root}")
        rec = {"path": d, "mount_path": v.get("mount_path"), "capacity": v.get("capacity"),
               "storage_class": v.get("storage_class")}
        repo = v.get("data_repository") or {}
        if repo.get("import_path") and repo.get("auto_import", True) and os.path.isdir(repo["import_path"]):
            rec["import"] = sync_tree(repo["import_path"], d)
        report["volumes"][v["name"]] = rec
    for h in cfg.get("home_dirs") or []:
        os.makedirs(os.path.join(root, h["volume"], h.get("path", "home")), exist_ok=True)
    for p in cfg.get("profiles") or []:
        pr.create(p["name"], owner=p.get("owner", "user@example.com"), gpu_quota=p.get("gpu_quota"),
                  contributors=p.get("contributors", []))
        report["profiles"].append(p["name"])
    os.makedirs(mxtrain_home(), exist_ok=True)
    with open(os.path.join(mxtrain_home(), "node.yaml"), "w") as f:
        yaml.safe_dump(dict(cfg, pv_root=root), f, sort_keys=False)
    return report


def applied_config() -> dict:
    p = os.path.join(mxtrain_home(), "node.yaml")
    if os.path.exists(p):
        with open(p) as f:
            return yaml.safe_load(f) or {}
    return dict(DEFAULT_CONFIG)


def stage_data(src: str, dest: str) -> Dict[str, int]:
    """src dir -> ``<claim>:<path>`` (the reference's stage-data pod: ``aws s3 cp
    --recursive s3://... /fsx/...``)."""
    claim, _, sub = dest.partition(":")
    d = os.path.join(pv_root(), claim, sub.lstrip("/"))
    if not os.path.isdir(src):
        raise FileNotFoundError(src)
    return sync_tree(src, d)


def export_volume(name: str) -> Dict[str, int]:
    cfg = applied_config()
    for v in cfg.get("volumes") or []:
        if v["name"] == name:
            repo = (v.get("data_repository") or {}).get("import_path")
            if not repo:
                raise ValueError(f"volume {name} has no data_repository.import_path")
            return sync_tree(os.path.join(pv_root(), name), repo)
    raise KeyError(name)


def attach_info() -> List[dict]:
    cfg = applied_config()
    out = []
    for v in cfg.get("volumes") or []:
        out.append({"claim": v["name"], "mount_path": v.get("mount_path"),
                    "host_path": os.path.join(pv_root(), v["name"])})
    return out

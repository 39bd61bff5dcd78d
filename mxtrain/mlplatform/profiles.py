"""Profiles (namespaces), GPU quotas and PodDefaults for the single-node launcher.

Replaces, for one MI355X node, the multi-user layer of the reference's Kubeflow platform:

* Profile controller + KFAM (C48, ``charts/ml-platform/kubeflow-profiles-and-kfam``,
  user profile ``kubeflow-user-example-com`` in
  ``charts/ml-platform/kubeflow-user-profile/templates/profile.yaml:1-15``): a profile is a
  namespace with an owner, contributors and a resource quota.
* Admission webhook PodDefaults (C50,
  ``charts/ml-platform/kubeflow-admission-webhook``) and the user-defaults PodDefault
  ``access-ml-pipeline`` (C30, ``charts/ml-platform/kubeflow-user-defaults/templates/
  pod_default.yaml:1-26``): label-selected env / volume injection into every replica the
  launcher starts in that namespace.
* Aggregated roles (C51): ``owner`` / ``contributor`` role per user, checked by
  ``can(user, verb, namespace)``.

State lives in ``$MXTRAIN_HOME/profiles/<namespace>.yaml`` (plain YAML, safe-loaded).
The launcher calls ``apply_pod_defaults`` for every replica and the GPU ledger calls
``gpu_quota`` before handing out devices (quota key ``amd.com/gpu``; the reference's
``nvidia.com/gpu`` is accepted as an alias).
"""
from __future__ import annotations

import os
import secrets
from typing import Dict, List, Optional

import yaml

from ..runtime.storage import mxtrain_home

DEFAULT_NS = "kubeflow-user-example-com"
QUOTA_KEYS = ("amd.com/gpu", "requests.amd.com/gpu", "nvidia.com/gpu", "requests.nvidia.com/gpu")


def profiles_dir() -> str:
    return os.path.join(mxtrain_home(), "profiles")


def _path(ns: str) -> str:
    return os.path.join(profiles_dir(), f"{ns}.yaml")


def _default_profile(ns: str) -> dict:
    """The reference's default user profile with its access-ml-pipeline PodDefault."""
    token_dir = os.path.join(profiles_dir(), ns, "pipelines-token")
    return {
        "apiVersion": "kubeflow.org/v1", "kind": "Profile",
        "metadata": {"name": ns},
        "spec": {
            "owner": {"kind": "User", "name": "user@example.com"},
            "contributors": [],
            "resourceQuotaSpec": {"hard": {}},
        },
        "podDefaults": [{
            "name": "access-ml-pipeline",
            "desc": "Allow access to the pipeline runner (mxtrain pipeline) from this namespace",
            "selector": {"matchLabels": {"access-ml-pipeline": "true"}},
            "env": [{"name": "KF_PIPELINES_SA_TOKEN_PATH",
                     "value": os.path.join(token_dir, "token")}],
            "volumes": [], "volumeMounts": [],
        }],
    }


def load(ns: str, create: bool = True) -> Optional[dict]:
    p = _path(ns)
    if os.path.exists(p):
        with open(p) as f:
            return yaml.safe_load(f) or {}
    if not create:
        return None
    prof = _default_profile(ns)
    save(prof)
    return prof


def save(prof: dict) -> str:
    ns = prof["metadata"]["name"]
    os.makedirs(profiles_dir(), exist_ok=True)
    for pd in prof.get("podDefaults") or []:
        for e in pd.get("env") or []:
            if e.get("name") == "KF_PIPELINES_SA_TOKEN_PATH":
                tp = e["value"]
                if not os.path.exists(tp):
                    os.makedirs(os.path.dirname(tp), exist_ok=True)
                    with open(tp, "w") as f:
                        f.write(secrets.token_hex(32))
                    os.chmod(tp, 0o600)
    tmp = _path(ns) + ".tmp"
    with open(tmp, "w") as f:
        yaml.safe_dump(prof, f, sort_keys=False)
    os.replace(tmp, _path(ns))
    return _path(ns)


def create(ns: str, owner: str = "user@example.com", gpu_quota: Optional[int] = None,
           contributors: List[str] = ()) -> dict:
    prof = load(ns, create=False) or _default_profile(ns)
    prof["spec"]["owner"] = {"kind": "User", "name": owner}
    prof["spec"]["contributors"] = [{"kind": "User", "name": c} for c in contributors]
    hard = prof["spec"].setdefault("resourceQuotaSpec", {}).setdefault("hard", {})
    if gpu_quota is not None:
        hard["amd.com/gpu"] = int(gpu_quota)
    save(prof)
    return prof


def delete(ns: str):
    p = _path(ns)
    if os.path.exists(p):
        os.remove(p)


def list_profiles() -> List[dict]:
    if not os.path.isdir(profiles_dir()):
        return []
    out = []
    for fn in sorted(os.listdir(profiles_dir())):
        if fn.endswith(".yaml"):
            with open(os.path.join(profiles_dir(), fn)) as f:
                out.append(yaml.safe_load(f) or {})
    return out


# ----------------------------------------------------------------------- quota / roles
def gpu_quota(ns: str) -> Optional[int]:
    prof = load(ns, create=False)
    if not prof:
        return None
    hard = ((prof.get("spec") or {}).get("resourceQuotaSpec") or {}).get("hard") or {}
    for k in QUOTA_KEYS:
        if k in hard and hard[k] not in (None, ""):
            return int(hard[k])
    return None


def can(user: str, verb: str, ns: str) -> bool:
    """owner: everything; contributor: create/get/list/delete jobs (KFAM 'edit')."""
    prof = load(ns, create=False)
    if not prof:
        return False
    spec = prof.get("spec") or {}
    if (spec.get("owner") or {}).get("name") == user:
        return True
    contributors = {c.get("name") for c in spec.get("contributors") or []}
    return user in contributors and verb in ("create", "get", "list", "delete", "logs")


# ----------------------------------------------------------------------- PodDefaults
def set_pod_default(ns: str, pd: dict) -> dict:
    prof = load(ns)
    pds = [p for p in prof.get("podDefaults") or [] if p.get("name") != pd.get("name")]
    pds.append(pd)
    prof["podDefaults"] = pds
    save(prof)
    return prof


def _matches(selector: dict, labels: Dict[str, str]) -> bool:
    ml = (selector or {}).get("matchLabels") or {}
    for k, v in ml.items():
        if str(labels.get(k)) != str(v):
            return False
    for expr in (selector or {}).get("matchExpressions") or []:
        k, op, vals = expr.get("key"), expr.get("operator"), [str(x) for x in expr.get("values") or []]
        have = k in labels
        if op == "In" and (not have or str(labels[k]) not in vals):
            return False
        if op == "NotIn" and have and str(labels[k]) in vals:
            return False
        if op == "Exists" and not have:
            return False
        if op == "DoesNotExist" and have:
            return False
    return bool(ml) or bool((selector or {}).get("matchExpressions"))


def matching_pod_defaults(ns: str, labels: Dict[str, str]) -> List[dict]:
    prof = load(ns, create=False)
    if not prof:
        return []
    return [pd for pd in prof.get("podDefaults") or [] if _matches(pd.get("selector"), labels or {})]


def apply_pod_defaults(ns: str, pod_template: dict, container: dict) -> List[str]:
    """Mutate ``container`` (env / volumeMounts) and the template's volumes the way the
    PodDefault admission webhook does: existing container settings win.  Returns the names
    of the applied PodDefaults (recorded in the replica's status)."""
    meta = pod_template.get("metadata") or {}
    # the reference's job templates carry app.kubernetes.io/* as annotations, not labels
    # (ml.annotations in every training chart): they count as labels for selection here
    labels = {k: v for k, v in (meta.get("annotations") or {}).items() if k.startswith("app.kubernetes.io/")}
    labels.update(meta.get("labels") or {})
    applied = []
    for pd in matching_pod_defaults(ns, labels):
        env = container.setdefault("env", [])
        have = {e.get("name") for e in env}
        for e in pd.get("env") or []:
            if e.get("name") not in have:
                env.append(dict(e))
        spec = pod_template.setdefault("spec", {})
        vols = spec.setdefault("volumes", [])
        vnames = {v.get("name") for v in vols}
        for v in pd.get("volumes") or []:
            if v.get("name") not in vnames:
                vols.append(dict(v))
        vms = container.setdefault("volumeMounts", [])
        mps = {m.get("mountPath") for m in vms}
        for m in pd.get("volumeMounts") or []:
            if m.get("mountPath") not in mps:
                vms.append(dict(m))
        applied.append(pd.get("name"))
    return applied

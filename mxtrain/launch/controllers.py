"""Job controllers: PyTorchJob (static + elastic), MPIJob, RayJob, Pod, Deployment.

Single-node replacements of the Kubeflow training-operator, mpi-operator and kuberay
(SURVEY §2.1 C20/C21/C21b, §3.1-§3.5, §5.3):

* PyTorchJob -- Master + Worker replicas (or Worker-only elastic), every replica gets the
  training-operator's env contract (PET_NNODES / PET_NPROC_PER_NODE / PET_NODE_RANK /
  PET_MASTER_ADDR / PET_MASTER_PORT, or PET_RDZV_* for elastic), HOSTNAME
  `pytorchjob-<rel>-master-0` / `-worker-<i>`, and a disjoint MI355X set (nproc_per_node
  GPUs) through HIP_VISIBLE_DEVICES.  restartPolicy OnFailure + runPolicy.backoffLimit are
  honoured as gang restarts; cleanPodPolicy Running stops the survivors when the job ends.
  With elasticPolicy the job is elastic instead (ElasticPyTorchJobController): hosted
  c10d rendezvous, per-replica restarts, min/max membership, scaling.
* MPIJob -- the launcher's `mpirun ... /etc/config/train-script.sh` runs through
  mxtrain.launch.mpirun (no ssh, no OpenMPI): np ranks on the worker replicas' slots.
* RayJob -- head group + worker group are realised as a GPU pool; the entrypoint runs as
  the driver with MXTRAIN_RAY_* env that mxtrain.raylike consumes.
* Pod / Deployment -- data-prep and testing charts.
"""
from __future__ import annotations

import json
import os
import socket
import time
from typing import Dict, List, Optional, Tuple

from ..runtime import affinity
from ..runtime.topology import GPUAllocator, gpus_requested
from .pods import Pod, build_pod, materialize_configmaps, python_exe

POLL = 0.25


def free_port(preferred: Optional[int] = None) -> int:
    if preferred:
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", int(preferred)))
            s.close()
            return int(preferred)
        except OSError:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class JobController:
    kind = "Job"

    def __init__(self, manifest: dict, manifests: List[dict], reldir: str, release: str,
                 allocator: GPUAllocator, status_cb=None):
        self.m = manifest
        self.manifests = manifests
        self.reldir = reldir
        self.release = release
        self.alloc = allocator
        self.status_cb = status_cb
        self.pods: List[Pod] = []
        self.phase = "Pending"
        self.restarts = 0
        self.message = ""
        self.cm_dirs = materialize_configmaps(manifests, reldir)
        self.gpus: List[int] = []
        self.mounts: Dict[str, str] = {}

    @property
    def name(self):
        return self.m.get("metadata", {}).get("name", self.kind.lower())

    # -- to implement
    def create_pods(self) -> List[Pod]:
        raise NotImplementedError

    def done(self) -> Optional[str]:
        """Return 'Succeeded' / 'Failed' when the job is finished, else None."""
        raise NotImplementedError

    # -- common machinery
    def backoff_limit(self) -> int:
        rp = (self.m.get("spec") or {}).get("runPolicy") or {}
        return int(rp.get("backoffLimit", 0) or 0)

    def restartable(self, pod: Pod) -> bool:
        return pod.spec.restart_policy in ("OnFailure", "Always")

    def status(self) -> dict:
        st = {"kind": self.kind, "name": self.name, "phase": self.phase, "restarts": self.restarts,
              "message": self.message, "gpus": self.gpus, "mounts": self.mounts,
              "pods": {p.spec.name: p.to_status() for p in self.pods}}
        pl = self.placement()
        if pl:
            st["placement"] = pl
        return st

    def placement(self) -> Optional[dict]:
        """Per-rank CPU/NUMA placement (rank -> gpu, numa node, cpuset)."""
        return getattr(self, "_placement", None)

    def place(self, gpu_sets: List[List[int]]) -> List[Tuple[List[int], Dict[str, str]]]:
        """NUMA-local cpusets for replicas that drive ``gpu_sets`` (one rank per GPU):
        returns per replica (cpuset of the replica = union of its ranks', env carrying the
        per-LOCAL_RANK sets).  Policy: MXTRAIN_CPU_BIND (core|numa|none)."""
        pol = affinity.default_bind()
        flat = [g for s in gpu_sets for g in s]
        if pol == "none" or not flat:
            return [([], {}) for _ in gpu_sets]
        pls = affinity.plan(flat, pol)
        self._placement = {"bind_to": pol, "ranks": [p.to_json() for p in pls]}
        out, i = [], 0
        for s in gpu_sets:
            mine = pls[i:i + len(s)]
            i += len(s)
            out.append((sorted({c for p in mine for c in p.cpus}), affinity.rank_env(mine) if mine else {}))
        return out

    def _emit(self):
        if self.status_cb:
            self.status_cb(self)

    def start(self):
        self.pods = self.create_pods()
        for p in self.pods:
            p.start()
        self.phase = "Running"
        self._emit()

    def stop(self):
        for p in self.pods:
            p.kill()

    def release_gpus(self):
        if self.gpus:
            self.alloc.release(self.gpus)
            self.gpus = []

    def step(self) -> bool:
        """One reconcile pass; returns True while the job is active."""
        for p in self.pods:
            p.poll()
        verdict = self.done()
        if verdict is None:
            # a failed restartable replica -> gang restart within the backoff budget
            failed = [p for p in self.pods if p.phase == "Failed"]
            if failed:
                if all(self.restartable(p) for p in failed) and self.restarts < self.backoff_limit():
                    self.restarts += 1
                    self.message = f"replica {failed[0].spec.name} failed (rc={failed[0].returncode}); restart {self.restarts}"
                    for p in self.pods:
                        p.kill()
                    self._on_restart()
                    for p in self.pods:
                        p.restarts = self.restarts
                        p.start()
                else:
                    verdict = "Failed"
                    self.message = f"replica {failed[0].spec.name} failed (rc={failed[0].returncode})"
        if verdict is not None:
            self.phase = verdict
            # cleanPodPolicy Running: stop replicas that are still alive
            for p in self.pods:
                p.kill()
            self.release_gpus()
            self._emit()
            return False
        self._emit()
        return True

    def _on_restart(self):
        pass


# ============================================================================ PyTorchJob
class PyTorchJobController(JobController):
    kind = "PyTorchJob"

    def _replicas(self):
        specs = (self.m.get("spec") or {}).get("pytorchReplicaSpecs") or {}
        out = []
        for role in ("Master", "Worker"):
            rs = specs.get(role)
            if rs:
                out.append((role, int(rs.get("replicas", 1) or 0), rs))
        return out

    def _nproc(self, tmpl) -> int:
        v = (self.m.get("spec") or {}).get("nprocPerNode")
        c = ((tmpl.get("spec") or {}).get("containers") or [{}])[0]
        req = gpus_requested(c.get("resources"))
        if v in (None, "", "auto", "gpu", "None"):
            return max(req, 1)
        if v == "cpu":
            return 1
        return int(v)

    def create_pods(self):
        reps = self._replicas()
        nnodes = sum(n for _, n, _ in reps)
        self.master_port = free_port()
        pods = []
        node_rank = 0
        sets = []
        for role, n, rs in reps:
            nproc = self._nproc(rs.get("template") or {})
            for i in range(n):
                gpus = self.alloc.allocate(nproc) if self.alloc.total > 0 else []
                self.gpus += gpus
                sets.append(gpus)
        placed = self.place(sets)
        for role, n, rs in reps:
            tmpl = rs.get("template") or {}
            nproc = self._nproc(tmpl)
            for i in range(n):
                gpus = sets[node_rank]
                cpus, penv = placed[node_rank]
                env = {"PET_NPROC_PER_NODE": str(nproc), "PET_NODE_RANK": str(node_rank),
                       "PET_MASTER_ADDR": "127.0.0.1", "PET_MASTER_PORT": str(self.master_port),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(self.master_port),
                       "WORLD_SIZE": str(nnodes), "RANK": str(node_rank), "PET_NNODES": str(nnodes)}
                name = f"{self.name}-{role.lower()}-{i}"
                env.update(penv)
                spec, plan = build_pod(name, tmpl, self.reldir, self.cm_dirs, env, gpus,
                                       rs.get("restartPolicy", "Never"), role=role, index=i)
                spec.cpus = cpus
                self.mounts.update(plan.mounts)
                pods.append(Pod(spec))
                node_rank += 1
        return pods

    def done(self):
        masters = [p for p in self.pods if p.spec.role == "Master"]
        if masters:
            if masters[0].phase == "Succeeded":
                return "Succeeded"
        elif self.pods and all(p.phase == "Succeeded" for p in self.pods):
            return "Succeeded"
        return None


# ============================================================================ elastic PyTorchJob
class ElasticPyTorchJobController(PyTorchJobController):
    """PyTorchJob with ``elasticPolicy`` (reference: charts/machine-learning/training/
    pytorchjob-elastic/templates/train.yaml:59-64; training-operator CRD
    crds/pytorchjobs.yaml:40-60).  Semantics, split as in Kubernetes between the
    operator and the torchrun elastic agent inside every replica:

    * the controller hosts the c10d rendezvous store (a TCPStore on ``rdzvPort``, so the
      rendezvous survives any replica) and hands every replica ``PET_NNODES=min:max``,
      ``PET_RDZV_*``, ``PET_MAX_RESTARTS=maxRestarts`` and ``PET_RDZV_CONF`` (+is_host=false);
    * a failing *worker process* is the agent's business: torchrun restarts its worker
      group (up to maxRestarts) and every agent re-rendezvouses, so the job re-forms
      without the operator touching the other replicas;
    * a failing *replica* (the agent itself exits non-zero) is restarted alone while the
      job's restart count is under ``runPolicy.backoffLimit`` -- no gang restart; once the
      budget is spent the replica stays down and the job continues while at least
      ``minReplicas`` replicas are alive;
    * membership changes between min and max with ``mxtrain scale <release> --replicas N``
      (``<reldir>/scale.json``): new replicas join at the next rendezvous round, removed
      ones leave and the survivors re-form;
    * the job succeeds when its replicas have exited and at least one succeeded (torchrun
      agents finish together); it fails when fewer than minReplicas remain.
    """

    def _policy(self):
        ep = (self.m.get("spec") or {}).get("elasticPolicy") or {}
        role, n, rs = [r for r in self._replicas() if r[0] == "Worker"][0]
        self.rs = rs
        self.min = int(ep.get("minReplicas") or n or 1)
        self.max = max(int(ep.get("maxReplicas") or max(n, self.min)), self.min)
        self.want = min(max(n, self.min), self.max)
        self.ep = ep

    def _host_store(self):
        from datetime import timedelta
        from torch.distributed import TCPStore
        last = None
        for port in (self.ep.get("rdzvPort"), 0):
            try:
                self.store = TCPStore("127.0.0.1", int(port or 0), is_master=True, multi_tenant=True,
                                      wait_for_workers=False, timeout=timedelta(seconds=600))
                self.rdzv_port = self.store.port
                return
            except (RuntimeError, ValueError) as e:   # preferred port busy -> any port
                last = e
        raise RuntimeError(f"cannot host the rendezvous store: {last}")

    def _rdzv_conf(self) -> str:
        kv = {}
        for item in self.ep.get("rdzvConf") or []:
            if isinstance(item, dict) and "key" in item:
                kv[str(item["key"])] = str(item.get("value", ""))
        kv["is_host"] = "false"
        return ",".join(f"{k}={v}" for k, v in kv.items())

    def _worker(self, index: int) -> Pod:
        tmpl = self.rs.get("template") or {}
        nproc = self._nproc(tmpl)
        gpus = self.alloc.allocate(nproc) if self.alloc.total > 0 else []
        self.gpus += gpus
        (cpus, penv), = self.place([gpus])
        nn = f"{self.min}:{self.max}" if self.min != self.max else str(self.min)
        env = {"PET_NNODES": nn, "PET_NPROC_PER_NODE": str(nproc), "PET_NODE_RANK": str(index),
               "PET_RDZV_BACKEND": str(self.ep.get("rdzvBackend", "c10d")),
               "PET_RDZV_ENDPOINT": f"127.0.0.1:{self.rdzv_port}",
               "PET_RDZV_ID": str(self.ep.get("rdzvId", self.release)),
               "PET_RDZV_CONF": self._rdzv_conf(), "PET_LOCAL_ADDR": "127.0.0.1",
               "PET_MAX_RESTARTS": str(self.ep.get("maxRestarts", 3)),
               "MASTER_ADDR": "127.0.0.1",
               # the agents' shared bootstrap store is built once per agent, in its first
               # round: a replica joining a later round then waits forever for a
               # MASTER_ADDR the round's rank 0 never republishes -> publish every round
               "TORCH_DISABLE_SHARE_RDZV_TCP_STORE": "1"}
        env.update(penv)
        spec, plan = build_pod(f"{self.name}-worker-{index}", tmpl, self.reldir, self.cm_dirs, env, gpus,
                               self.rs.get("restartPolicy", "Never"), role="Worker", index=index)
        spec.cpus = cpus
        self.mounts.update(plan.mounts)
        return Pod(spec)

    def create_pods(self):
        self._policy()
        self._host_store()
        self.down: List[str] = []        # replicas out of the job (budget spent / scaled down)
        self.next_index = self.want
        self._scale_mtime = None
        return [self._worker(i) for i in range(self.want)]

    def status(self):
        st = super().status()
        if not hasattr(self, "down"):
            return st
        st["elastic"] = {"minReplicas": self.min, "maxReplicas": self.max, "replicas": len(self._live()),
                         "rdzvEndpoint": f"127.0.0.1:{getattr(self, 'rdzv_port', None)}", "removed": self.down}
        return st

    def _live(self) -> List[Pod]:
        return [p for p in self.pods if p.spec.name not in self.down]

    def _drop(self, pod: Pod, why: str):
        pod.kill()
        self.down.append(pod.spec.name)
        if pod.spec.gpus:
            self.alloc.release(pod.spec.gpus)
            self.gpus = [g for g in self.gpus if g not in pod.spec.gpus]
        self.message = why

    def _rescale(self):
        path = os.path.join(self.reldir, "scale.json")
        try:
            mt = os.path.getmtime(path)
        except OSError:
            return
        if mt == self._scale_mtime:
            return
        self._scale_mtime = mt
        try:
            with open(path) as f:
                n = int(json.load(f)["replicas"])
        except (OSError, ValueError, KeyError, TypeError):
            return
        n = min(max(n, self.min), self.max)
        live = [p for p in self._live() if p.phase in ("Running", "Pending")]
        while len(live) < n:
            try:
                p = self._worker(self.next_index)
            except RuntimeError as e:    # no GPU free -> stay at the current size
                self.message = f"scale to {n}: {e}"
                break
            self.next_index += 1
            p.start()
            self.pods.append(p)
            live.append(p)
            self.message = f"scaled up: {p.spec.name} joins at the next rendezvous"
        for p in sorted(live, key=lambda q: -q.spec.index)[:max(0, len(live) - n)]:
            self._drop(p, f"scaled down: {p.spec.name} removed, survivors re-form")

    def step(self) -> bool:
        for p in self.pods:
            p.poll()
        self._rescale()
        for p in self._live():
            if p.phase != "Failed":
                continue
            if self.restartable(p) and self.restarts < self.backoff_limit():
                self.restarts += 1
                p.restarts += 1
                self.message = (f"replica {p.spec.name} failed (rc={p.returncode}); restarting it alone "
                                f"({self.restarts}/{self.backoff_limit()}), it rejoins the rendezvous")
                p.start()
            else:
                self._drop(p, f"replica {p.spec.name} failed (rc={p.returncode}); restart budget spent")
        live = self._live()
        verdict = None
        if len(live) < self.min and not any(p.phase == "Succeeded" for p in live):
            verdict = "Failed"
            self.message = (f"{len(live)} replica(s) alive < minReplicas={self.min}" +
                            (f"; {self.message}" if self.message else ""))
        elif live and all(p.phase in ("Succeeded", "Failed") for p in live) and \
                any(p.phase == "Succeeded" for p in live):
            verdict = "Succeeded"
        if verdict is not None:
            self.phase = verdict
            for p in self.pods:
                p.kill()
            self.release_gpus()
            self._stop_store()
            self._emit()
            return False
        self._emit()
        return True

    def stop(self):
        super().stop()
        self._stop_store()

    def _stop_store(self):
        self.store = None


def _pytorchjob(manifest, *a, **kw):
    if (manifest.get("spec") or {}).get("elasticPolicy"):
        return ElasticPyTorchJobController(manifest, *a, **kw)
    return PyTorchJobController(manifest, *a, **kw)


# ============================================================================ MPIJob
class MPIJobController(JobController):
    kind = "MPIJob"

    def create_pods(self):
        spec = self.m.get("spec") or {}
        rs = spec.get("mpiReplicaSpecs") or {}
        worker = rs.get("Worker") or {}
        launcher = rs.get("Launcher") or {}
        nworkers = int(worker.get("replicas", 1) or 1)
        slots = int(spec.get("slotsPerWorker", 1) or 1)
        wt = worker.get("template") or {}
        per_worker_gpus = gpus_requested(((wt.get("spec") or {}).get("containers") or [{}])[0].get("resources"))
        per_worker_gpus = per_worker_gpus or (slots if self.alloc.total else 0)
        worker_sets = []
        for i in range(nworkers):
            g = self.alloc.allocate(min(per_worker_gpus, slots) if per_worker_gpus else 0) \
                if self.alloc.total else []
            self.gpus += g
            worker_sets.append(g)
        # resolve the worker pod (env, volumes, mounts) once; ranks inherit it
        wspec, wplan = build_pod(f"{self.name}-worker-0", wt, self.reldir, self.cm_dirs, {}, [],
                                 "Never", role="Worker")
        self.mounts.update(wplan.mounts)
        wfile = os.path.join(self.reldir, "mpi-workers.json")
        with open(wfile, "w") as f:
            json.dump({"workers": [{"name": f"{self.name}-worker-{i}", "gpus": worker_sets[i]}
                                   for i in range(nworkers)],
                       "slots": slots, "env": {k: v for k, v in wspec.env.items()
                                               if k not in os.environ or os.environ[k] != v},
                       "workdir": wspec.workdir, "mounts": wplan.mounts,
                       "mount_mode": wplan.mode}, f, indent=1)
        lt = launcher.get("template") or {}
        lc = ((lt.get("spec") or {}).get("containers") or [{}])[0]
        cmd = list(lc.get("command") or []) + list(lc.get("args") or [])
        if cmd and os.path.basename(cmd[0]) == "mpirun":
            cmd = [python_exe(), "-m", "mxtrain.launch.mpirun"] + cmd[1:]
        self.placement_file = os.path.join(self.reldir, "mpi-placement.json")
        env = {"MXTRAIN_MPI_WORKERS": wfile, "MXTRAIN_MPI_SLOTS": str(slots),
               "MXTRAIN_MPI_PLACEMENT": self.placement_file}
        # the launcher has no PVCs in the reference; resolve paths with the workers' plan
        lspec, _ = build_pod(f"{self.name}-launcher", lt, self.reldir, self.cm_dirs, env, [],
                             (lt.get("spec") or {}).get("restartPolicy", "OnFailure"),
                             command_override=cmd, role="Launcher")
        lspec.command = [wplan.rewrite(x) for x in lspec.command]
        for k, v in list(lspec.env.items()):
            lspec.env[k] = wplan.rewrite(v)
        return [Pod(lspec)]

    def done(self):
        p = self.pods[0]
        if p.phase == "Succeeded":
            return "Succeeded"
        return None

    def placement(self):
        try:
            with open(self.placement_file) as f:
                return json.load(f)
        except (AttributeError, OSError, ValueError):
            return None


# ============================================================================ RayJob
class RayJobController(JobController):
    kind = "RayJob"

    def create_pods(self):
        spec = self.m.get("spec") or {}
        rc = spec.get("rayClusterSpec") or {}
        head = (rc.get("headGroupSpec") or {}).get("template") or {}
        groups = rc.get("workerGroupSpecs") or []
        ngpu = 0
        nworkers = 0
        for g in groups:
            reps = int(g.get("replicas", 1) or 0)
            c = (((g.get("template") or {}).get("spec") or {}).get("containers") or [{}])[0]
            ngpu += reps * gpus_requested(c.get("resources"))
            nworkers += reps
        gpus = self.alloc.allocate(min(ngpu, self.alloc.total)) if (ngpu and self.alloc.total) else []
        self.gpus = gpus
        # one Ray Train worker per GPU of the worker group (CPU groups: one per replica)
        env = {"MXTRAIN_RAY_NUM_WORKERS": str(len(gpus) if gpus else max(nworkers, 1)),
               "MXTRAIN_RAY_GPUS": ",".join(str(x) for x in gpus),
               "RAY_ADDRESS": "mxtrain://127.0.0.1", "MXTRAIN_RAY_JOB": self.release}
        rt = spec.get("runtimeEnvYAML")
        if rt:
            import yaml
            renv = yaml.safe_load(rt) or {}
            for k, v in (renv.get("env_vars") or {}).items():
                env[k] = str(v)
            if renv.get("pip"):
                env["MXTRAIN_RAY_PIP_IGNORED"] = json.dumps(renv.get("pip"))
        entry = spec.get("entrypoint") or ""
        cmd = ["bash", "-c", entry] if entry else []
        (cpus, penv), = self.place([gpus])
        env.update(penv)
        pspec, plan = build_pod(f"rayjob-{self.release}-submitter", head, self.reldir, self.cm_dirs,
                                env, gpus, "Never", command_override=cmd, role="Submitter")
        pspec.cpus = cpus
        # the entrypoint is a shell line; rewrite mount prefixes inside it as well
        pspec.command = [plan.rewrite(x) for x in pspec.command]
        self.mounts.update(plan.mounts)
        return [Pod(pspec)]

    def done(self):
        return "Succeeded" if self.pods[0].phase == "Succeeded" else None


# ============================================================================ Pod / Deployment
class PodController(JobController):
    kind = "Pod"

    def create_pods(self):
        spec = self.m.get("spec") or {}
        c = (spec.get("containers") or [{}])[0]
        n = gpus_requested(c.get("resources"))
        gpus = self.alloc.allocate(n) if (n and self.alloc.total) else []
        self.gpus = gpus
        (cpus, penv), = self.place([gpus])
        pspec, plan = build_pod(self.name, {"spec": spec}, self.reldir, self.cm_dirs, penv, gpus,
                                spec.get("restartPolicy", "Always"))
        pspec.cpus = cpus
        self.mounts.update(plan.mounts)
        return [Pod(pspec)]

    def done(self):
        p = self.pods[0]
        return "Succeeded" if p.phase == "Succeeded" else None


class DeploymentController(JobController):
    kind = "Deployment"

    def create_pods(self):
        spec = self.m.get("spec") or {}
        tmpl = spec.get("template") or {}
        n = int(spec.get("replicas", 1) or 1)
        pods = []
        for i in range(n):
            for ci, c in enumerate((tmpl.get("spec") or {}).get("containers") or []):
                ng = gpus_requested(c.get("resources"))
                gpus = self.alloc.allocate(ng) if (ng and self.alloc.total) else []
                self.gpus += gpus
                pspec, plan = build_pod(f"{self.name}-{i}-{c.get('name', ci)}", tmpl, self.reldir,
                                        self.cm_dirs, {}, gpus, "Always", container_index=ci)
                self.mounts.update(plan.mounts)
                pods.append(Pod(pspec))
        return pods

    def backoff_limit(self):
        return 10

    def done(self):
        return None  # runs until uninstalled


CONTROLLERS = {"PyTorchJob": _pytorchjob, "MPIJob": MPIJobController,
               "RayJob": RayJobController, "Pod": PodController, "Deployment": DeploymentController}
PASSIVE_KINDS = {"ConfigMap", "Secret", "Service", "PersistentVolumeClaim", "PersistentVolume",
                 "StorageClass", "ServiceAccount"}

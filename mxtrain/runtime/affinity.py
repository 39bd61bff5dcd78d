"""Per-rank CPU / NUMA placement (SURVEY §7.1 decision 1; the reference leaves it to
OpenMPI's ``-bind-to`` / ``-map-by`` in ``mpijob-horovod-tensorflow-gpu/values.yaml:60-122``
and to the kubelet's CPU manager).

One rank drives one MI355X.  Its host threads (Python, the HIP runtime's submission
thread, data-loader workers) belong on the cores of the socket the GPU hangs off, and
ranks sharing a socket should not contend for the same cores.  This module

* reads which NUMA node every GPU is attached to from the KFD topology (GPU node ->
  PCI location -> ``/sys/bus/pci/devices/*/numa_node``; falls back to the KFD io_link
  to a CPU node), and each NUMA node's CPUs from ``/sys/devices/system/node``;
* plans disjoint, NUMA-local cpusets for a list of ranks (``plan``), honouring the
  OpenMPI binding vocabulary: ``core`` (default: an equal, disjoint slice of the local
  node's cores per rank), ``numa``/``socket``/``package`` (the whole local node),
  ``hwthread`` (one CPU), ``none`` (no pinning);
* applies a plan in the child (``preexec`` for ``subprocess.Popen``) or, for ranks
  started by torchrun inside a replica, from ``MXTRAIN_RANK_CPUSETS`` by LOCAL_RANK
  (``pin_self_from_env``, called by ``parallel.state.init_distributed``).

All sysfs reads go through ``root`` (default ``/``, or ``MXTRAIN_SYSFS_ROOT``) so tests
run against a fake topology.
"""
from __future__ import annotations

import glob
import json
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

BIND_MODES = ("none", "core", "hwthread", "numa", "socket", "package", "l3cache", "board")


def _root(root: Optional[str]) -> str:
    return root if root is not None else os.environ.get("MXTRAIN_SYSFS_ROOT", "/")


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def parse_cpulist(s: str) -> List[int]:
    """'0-3,8,10-11' -> [0,1,2,3,8,10,11]."""
    out: List[int] = []
    for part in (s or "").replace("\n", ",").split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(set(out))


def format_cpulist(cpus: Sequence[int]) -> str:
    cpus = sorted(set(cpus))
    runs, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        runs.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(runs)


def numa_cpus(root: Optional[str] = None) -> Dict[int, List[int]]:
    """NUMA node -> its online CPUs (nodes without CPUs are skipped)."""
    r = _root(root)
    out = {}
    for p in glob.glob(os.path.join(r, "sys/devices/system/node/node[0-9]*")):
        cl = _read(os.path.join(p, "cpulist"))
        cpus = parse_cpulist(cl) if cl else []
        if cpus:
            out[int(os.path.basename(p)[4:])] = cpus
    return dict(sorted(out.items()))


def _kfd_nodes(r: str) -> List[dict]:
    nodes = []
    for p in sorted(glob.glob(os.path.join(r, "sys/class/kfd/kfd/topology/nodes/*/properties")),
                    key=lambda q: int(q.split("/")[-2])):
        txt = _read(p) or ""
        props = {}
        for line in txt.splitlines():
            kv = line.split()
            if len(kv) == 2:
                props[kv[0]] = kv[1]
        props["_id"] = int(p.split("/")[-2])
        props["_dir"] = os.path.dirname(p)
        nodes.append(props)
    return nodes


def gpu_numa_nodes(root: Optional[str] = None) -> List[int]:
    """NUMA node of every GPU, in the same (KFD enumeration) order as
    ``topology._kfd_gpus`` / HIP device ids; -1 if unknown."""
    r = _root(root)
    nodes = _kfd_nodes(r)
    cpu_nodes = [n["_id"] for n in nodes if int(n.get("cpu_cores_count", "0")) > 0
                 and int(n.get("gfx_target_version", "0")) == 0]
    out = []
    for n in nodes:
        if int(n.get("gfx_target_version", "0")) == 0:
            continue
        numa = -1
        loc = int(n.get("location_id", "-1"))
        if loc >= 0:
            dom = int(n.get("domain", "0"))
            bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}"
            v = _read(os.path.join(r, "sys/bus/pci/devices", bdf, "numa_node"))
            if v not in (None, "") and int(v) >= 0:
                numa = int(v)
        if numa < 0:
            # io_link to a CPU node: KFD numbers CPU nodes in NUMA order
            for lp in glob.glob(os.path.join(n["_dir"], "io_links/*/properties")):
                props = dict(line.split() for line in (_read(lp) or "").splitlines() if len(line.split()) == 2)
                to = int(props.get("node_to", "-1"))
                if to in cpu_nodes:
                    numa = cpu_nodes.index(to)
                    break
        out.append(numa)
    return out


def physical_cores(cpus: Sequence[int], root: Optional[str] = None) -> List[List[int]]:
    """Group CPUs into physical cores via ``topology/thread_siblings_list`` (each CPU is
    its own core when sysfs does not say), ordered by the first CPU of each core."""
    r = _root(root)
    cs = set(cpus)
    seen, out = set(), []
    for c in sorted(cs):
        if c in seen:
            continue
        sib = _read(os.path.join(r, f"sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list"))
        grp = [x for x in (parse_cpulist(sib) if sib else [c]) if x in cs] or [c]
        seen.update(grp)
        out.append(sorted(grp))
    return out


@dataclass
class Placement:
    rank: int
    gpu: Optional[int]
    numa: int
    cpus: List[int]

    def to_json(self) -> dict:
        return {"rank": self.rank, "gpu": self.gpu, "numa": self.numa, "cpus": format_cpulist(self.cpus)}


def plan(gpus: Sequence[Optional[int]], bind_to: str = "core", root: Optional[str] = None,
         allowed: Optional[Sequence[int]] = None) -> List[Placement]:
    """Cpusets for ranks 0..len(gpus)-1, rank i driving physical GPU ``gpus[i]`` (None =
    CPU-only rank).  Ranks are assigned to the NUMA node of their GPU; CPU-only ranks
    and GPUs of unknown locality are spread over the nodes round-robin.  ``allowed``
    restricts every cpuset (the launcher's own affinity by default)."""
    mode = (bind_to or "core").split(":")[0].lower()
    if mode not in BIND_MODES:
        raise ValueError(f"unsupported bind-to {bind_to!r} (one of {', '.join(BIND_MODES)})")
    allowed_set = set(allowed if allowed is not None else _self_affinity())
    nodes = {k: [c for c in v if c in allowed_set] for k, v in numa_cpus(root).items()}
    nodes = {k: v for k, v in nodes.items() if v}
    if not nodes:
        nodes = {0: sorted(allowed_set)}
    g2n = gpu_numa_nodes(root)
    order = sorted(nodes)
    ranks_numa = []
    rr = 0
    for g in gpus:
        n = g2n[g] if (g is not None and 0 <= g < len(g2n)) else -1
        if n not in nodes:
            n = order[rr % len(order)]
            rr += 1
        ranks_numa.append(n)
    out = []
    for n in order:
        members = [i for i, x in enumerate(ranks_numa) if x == n]
        cpus = nodes[n]
        if not members:
            continue
        if mode in ("numa", "socket", "package", "l3cache", "board", "none"):
            for i in members:
                out.append(Placement(i, gpus[i], n, list(cpus)))
            continue
        # core / hwthread: equal disjoint slices of the node's physical cores (SMT
        # siblings stay with their core); more ranks than cores wrap (oversubscribe)
        cores = physical_cores(cpus, root)
        k = len(members)
        per = max(1, len(cores) // k)
        for j, i in enumerate(members):
            if len(cores) >= k:
                grp = cores[j * per:(j + 1) * per]
            else:
                grp = [cores[j % len(cores)]]
            sl = sorted(c for core in grp for c in core)
            if mode == "hwthread":
                sl = sl[:1]
            out.append(Placement(i, gpus[i], n, sl))
    out.sort(key=lambda p: p.rank)
    return out


def _self_affinity() -> List[int]:
    try:
        return sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return list(range(os.cpu_count() or 1))


def default_bind() -> str:
    return os.environ.get("MXTRAIN_CPU_BIND", "core")


def preexec(cpus: Sequence[int]):
    """A ``Popen(preexec_fn=...)`` that pins the child before it execs."""
    cs = set(cpus)

    def fn():
        if cs:
            try:
                os.sched_setaffinity(0, cs)
            except OSError:
                pass
    return fn


def rank_env(placements: Sequence[Placement]) -> Dict[str, str]:
    """Env for a replica whose local ranks (torchrun LOCAL_RANK order) get these sets."""
    return {"MXTRAIN_RANK_CPUSETS": json.dumps([format_cpulist(p.cpus) for p in placements])}


def pin_self_from_env(local_rank: Optional[int] = None) -> Optional[List[int]]:
    """Pin the calling rank to ``MXTRAIN_RANK_CPUSETS[LOCAL_RANK]`` (set by the job
    controller for replicas that start several ranks themselves).  Returns the cpuset
    or None when no plan is present / pinning is off."""
    raw = os.environ.get("MXTRAIN_RANK_CPUSETS")
    if not raw or default_bind() == "none":
        return None
    sets = json.loads(raw)
    lr = int(os.environ.get("LOCAL_RANK", "0")) if local_rank is None else local_rank
    if not (0 <= lr < len(sets)):
        return None
    cpus = parse_cpulist(sets[lr])
    try:
        os.sched_setaffinity(0, set(cpus))
    except OSError:
        return None
    return cpus

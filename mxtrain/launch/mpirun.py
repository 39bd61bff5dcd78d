"""mpirun-compatible rank spawner (replaces OpenMPI launch + mpi-operator hostfile/ssh;
SURVEY §2.1 C04/C21, §2.2 "mpirun.args", §3.3, §7.1.3).

    python -m mxtrain.launch.mpirun [OpenMPI options] <program> [args...]

No ssh, no orted, no MPI library: the ranks of one node are children of this process.
Every rank gets the OpenMPI rank environment (OMPI_COMM_WORLD_{RANK,SIZE,LOCAL_RANK,
LOCAL_SIZE,NODE_RANK}, PMIX_RANK) *and* the torch.distributed env:// contract
(RANK/WORLD_SIZE/LOCAL_RANK/LOCAL_WORLD_SIZE/MASTER_ADDR/MASTER_PORT), so a Horovod-style
workload initialises RCCL directly (mxtrain.dist.hvd).

Supported options (the subset the reference's mpirun.args use, values.yaml:60-122):
  -np/-n/-c N, -x VAR[=VAL], --output-filename DIR, --tag-output, --timestamp-output,
  --display-map, --report-bindings, -bind-to/--bind-to X (none|core|hwthread|numa|socket),
  -map-by/--map-by X (slot|node|ppr:N:node),
  -H/--host, --hostfile, -mca/--mca K V (ignored, echoed with -v), --allow-run-as-root,
  --oversubscribe, -wdir/--wdir DIR.
Ranks are mapped onto the worker replicas of the MPIJob (MXTRAIN_MPI_WORKERS json written
by the controller): map-by slot fills worker 0's slots first, map-by node round-robins.
If any rank fails the others are terminated (OpenMPI's default abort semantics) and the
failing rank's exit code is returned.

Binding: every rank is pinned (sched_setaffinity before exec) to a cpuset on the NUMA node
of the GPU it drives (runtime.affinity): ``core`` = disjoint equal slices of that node,
``numa``/``socket`` = the whole node, ``none`` = unpinned.  Without ``-bind-to`` the policy
is ``MXTRAIN_CPU_BIND`` (default ``core``).  The placement is printed by --display-map /
--report-bindings and written to ``MXTRAIN_MPI_PLACEMENT`` (the controller puts it in the
job status).
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..runtime import affinity

FLAGS_WITH_ARG = {"-np", "-n", "-c", "--np", "-x", "--output-filename", "-output-filename",
                  "-bind-to", "--bind-to", "-map-by", "--map-by", "-H", "--host", "-host",
                  "--hostfile", "-hostfile", "--machinefile", "-wdir", "--wdir", "-rank-by",
                  "--rank-by", "--rankfile", "-npernode", "--npernode", "--prefix", "-N"}
FLAGS_WITH_TWO = {"-mca", "--mca", "-gmca", "--gmca"}


@dataclass
class MpirunArgs:
    np: Optional[int] = None
    exports: List[str] = field(default_factory=list)
    output_filename: Optional[str] = None
    tag_output: bool = False
    timestamp_output: bool = False
    display_map: bool = False
    map_by: str = "slot"
    bind_to: Optional[str] = None
    report_bindings: bool = False
    mca: Dict[str, str] = field(default_factory=dict)
    wdir: Optional[str] = None
    verbose: bool = False
    program: List[str] = field(default_factory=list)


def parse_args(argv: List[str]) -> MpirunArgs:
    a = MpirunArgs()
    i = 0
    while i < len(argv):
        t = argv[i]
        if not t.startswith("-") or t == "--":
            a.program = argv[i + 1:] if t == "--" else argv[i:]
            break
        if "=" in t and t.startswith("--") and t.split("=", 1)[0] in FLAGS_WITH_ARG:
            t, val = t.split("=", 1)
            argv = argv[:i] + [t, val] + argv[i + 1:]
        if t in FLAGS_WITH_TWO:
            a.mca[argv[i + 1]] = argv[i + 2]
            i += 3
            continue
        if t in FLAGS_WITH_ARG:
            v = argv[i + 1]
            if t in ("-np", "-n", "-c", "--np"):
                a.np = int(v)
            elif t == "-x":
                a.exports.append(v)
            elif t in ("--output-filename", "-output-filename"):
                # the pod spec passes "$HOME/logs/..." unexpanded; the intent is the
                # launcher's $HOME, so expand (an OpenMPI launcher would create "$HOME/")
                a.output_filename = os.path.expandvars(v)
            elif t in ("-map-by", "--map-by"):
                a.map_by = v
            elif t in ("-bind-to", "--bind-to"):
                a.bind_to = v
            elif t in ("-wdir", "--wdir"):
                a.wdir = os.path.expandvars(v)
            i += 2
            continue
        if t in ("--tag-output", "-tag-output"):
            a.tag_output = True
        elif t in ("--timestamp-output", "-timestamp-output"):
            a.timestamp_output = True
        elif t in ("--display-map", "-display-map"):
            a.display_map = True
        elif t in ("--report-bindings", "-report-bindings"):
            a.report_bindings = True
        elif t in ("-v", "--verbose"):
            a.verbose = True
        # --allow-run-as-root, --oversubscribe, -q ... are no-ops here
        i += 1
    if not a.program:
        raise SystemExit("mpirun: no executable specified")
    return a


def load_workers(slots_default: int) -> dict:
    path = os.environ.get("MXTRAIN_MPI_WORKERS")
    if path and os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    n = int(os.environ.get("MXTRAIN_MPI_SLOTS", slots_default))
    vis = os.environ.get("HIP_VISIBLE_DEVICES")
    gpus = [int(x) for x in vis.split(",")] if vis else []
    return {"workers": [{"name": os.environ.get("HOSTNAME", "localhost"), "gpus": gpus}], "slots": n,
            "env": {}, "workdir": None, "mounts": {}, "mount_mode": {}}


def rank_map(np_: int, nworkers: int, slots: int, map_by: str) -> List[int]:
    """rank -> worker index."""
    if map_by.startswith("ppr:"):
        per = int(map_by.split(":")[1])
        return [min(r // per, nworkers - 1) for r in range(np_)]
    if map_by.startswith("node"):
        return [r % nworkers for r in range(np_)]
    # slot (default): fill each worker's slots, wrap (oversubscribe) if np > total
    return [(r // slots) % nworkers for r in range(np_)]


def bind_policy(args: MpirunArgs) -> str:
    return (args.bind_to or affinity.default_bind()).lower()


def rank_placements(args: MpirunArgs, workers: List[dict], wmap: List[int]) -> List[Optional["affinity.Placement"]]:
    """rank -> Placement (None when unbound).  A rank drives GPU ``gpus[local_rank]`` of
    its worker (HIP_VISIBLE_DEVICES holds the worker's set, the rank picks by LOCAL_RANK)."""
    pol = bind_policy(args)
    if pol == "none":
        return [None] * len(wmap)
    gpus, counters = [], {}
    for w in wmap:
        lr = counters.get(w, 0)
        counters[w] = lr + 1
        g = workers[w].get("gpus") or []
        gpus.append(g[lr % len(g)] if g else None)
    return affinity.plan(gpus, pol)


def _bound(p) -> str:
    if p is None:
        return "N/A"
    return f"numa {p.numa}[cpus {affinity.format_cpulist(p.cpus)}]" + (f" gpu {p.gpu}" if p.gpu is not None else "")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Pump(threading.Thread):
    """Copies one rank stream to the launcher's stdout (tagged/timestamped) and to the
    OpenMPI-style per-rank file <output-filename>/1/rank.<r>/{stdout,stderr}."""

    def __init__(self, stream, rank: int, kind: str, args: MpirunArgs, out_lock: threading.Lock):
        super().__init__(daemon=True)
        self.stream, self.rank, self.kind, self.args, self.lock = stream, rank, kind, args, out_lock
        self.file = None
        if args.output_filename:
            d = os.path.join(args.output_filename, "1", f"rank.{rank}")
            os.makedirs(d, exist_ok=True)
            self.file = open(os.path.join(d, kind), "ab")

    def run(self):
        out = sys.stdout.buffer if self.kind == "stdout" else sys.stderr.buffer
        for line in iter(self.stream.readline, b""):
            if self.file:
                self.file.write(line)
                self.file.flush()
            prefix = b""
            if self.args.tag_output:
                prefix += f"[1,{self.rank}]<{self.kind}>:".encode()
            if self.args.timestamp_output:
                prefix = time.strftime("%a %b %d %H:%M:%S %Y").encode() + b", " + prefix
            with self.lock:
                out.write(prefix + line)
                out.flush()
        if self.file:
            self.file.close()


def build_rank_env(base: Dict[str, str], spec: dict, args: MpirunArgs, rank: int, np_: int,
                   worker: int, local_rank: int, local_size: int, port: int) -> Dict[str, str]:
    env = dict(base)
    env.update(spec.get("env") or {})
    for x in args.exports:
        if "=" in x:
            k, v = x.split("=", 1)
            env[k] = v
        elif x in base:
            env[x] = base[x]
    w = spec["workers"][worker]
    env["HOSTNAME"] = w.get("name", env.get("HOSTNAME", "localhost"))
    if w.get("gpus"):
        env["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in w["gpus"])
    env.update({
        "OMPI_COMM_WORLD_RANK": str(rank), "OMPI_COMM_WORLD_SIZE": str(np_),
        "OMPI_COMM_WORLD_LOCAL_RANK": str(local_rank), "OMPI_COMM_WORLD_LOCAL_SIZE": str(local_size),
        "OMPI_COMM_WORLD_NODE_RANK": str(worker), "PMIX_RANK": str(rank),
        "OMPI_UNIVERSE_SIZE": str(np_),
        "RANK": str(rank), "WORLD_SIZE": str(np_), "LOCAL_RANK": str(local_rank),
        "LOCAL_WORLD_SIZE": str(local_size), "GROUP_RANK": str(worker),
        "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
    })
    for k, v in args.mca.items():
        env[f"OMPI_MCA_{k}"] = v
    return env


def run(argv: List[str]) -> int:
    args = parse_args(argv)
    spec = load_workers(1)
    workers = spec["workers"]
    slots = int(spec.get("slots", 1))
    np_ = args.np if args.np is not None else slots * len(workers)
    wmap = rank_map(np_, len(workers), slots, args.map_by)
    local_sizes = {w: wmap.count(w) for w in set(wmap)}
    port = _free_port()
    placements = rank_placements(args, workers, wmap)
    ppath = os.environ.get("MXTRAIN_MPI_PLACEMENT")
    if ppath:
        with open(ppath, "w") as f:
            json.dump({"bind_to": bind_policy(args), "map_by": args.map_by,
                       "ranks": [p.to_json() if p else None for p in placements]}, f, indent=1)
    if args.display_map:
        print(" ========================   JOB MAP   ========================")
        for wi, w in enumerate(workers):
            ranks = [r for r in range(np_) if wmap[r] == wi]
            print(f"\n Data for node: {w.get('name')}\tNum slots: {slots}\tNum procs: {len(ranks)}")
            for r in ranks:
                print(f" \tProcess OMPI jobid: [1,0] App: 0 Process rank: {r} Bound: {_bound(placements[r])}")
        print("\n =============================================================", flush=True)
    if args.report_bindings:
        for r, p in enumerate(placements):
            sys.stderr.write(f"[mxtrain-mpirun] MCW rank {r} bound to {_bound(p)}\n")
    base = dict(os.environ)
    procs: List[subprocess.Popen] = []
    pumps: List[_Pump] = []
    lock = threading.Lock()
    prog = list(args.program)
    if prog[0].endswith(".sh") and os.path.isfile(prog[0]) and not os.access(prog[0], os.X_OK):
        prog = ["bash"] + prog
    counters: Dict[int, int] = {}
    for r in range(np_):
        w = wmap[r]
        lr = counters.get(w, 0)
        counters[w] = lr + 1
        env = build_rank_env(base, spec, args, r, np_, w, lr, local_sizes[w], port)
        cwd = args.wdir or spec.get("workdir") or os.getcwd()
        if not os.path.isdir(cwd):
            cwd = os.getcwd()
        pl = placements[r]
        p = subprocess.Popen(prog, env=env, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             start_new_session=True, preexec_fn=affinity.preexec(pl.cpus) if pl else None)
        procs.append(p)
        for stream, kind in ((p.stdout, "stdout"), (p.stderr, "stderr")):
            t = _Pump(stream, r, kind, args, lock)
            t.start()
            pumps.append(t)

    def _terminate(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except ProcessLookupError:
                    pass

    def _on_signal(signum, frame):
        _terminate()
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, _on_signal)
    signal.signal(signal.SIGINT, _on_signal)
    rc = 0
    failed_rank = None
    while True:
        alive = False
        for r, p in enumerate(procs):
            c = p.poll()
            if c is None:
                alive = True
            elif c != 0 and failed_rank is None:
                failed_rank, rc = r, c
        if failed_rank is not None:
            _terminate()
            t0 = time.time()
            while any(p.poll() is None for p in procs) and time.time() - t0 < 10:
                time.sleep(0.1)
            _terminate(signal.SIGKILL)
            break
        if not alive:
            break
        time.sleep(0.1)
    for p in procs:
        p.wait()
    for t in pumps:
        t.join(timeout=5)
    if failed_rank is not None:
        sys.stderr.write(
            "--------------------------------------------------------------------------\n"
            f"Primary job  terminated normally, but 1 process returned\na non-zero exit code. "
            f"Per user-direction, the job has been aborted.\n"
            f"mpirun detected that one or more processes exited with non-zero status, thus causing\n"
            f"the job to be terminated. The first process to do so was:\n\n"
            f"  Process name: [[1,0],{failed_rank}]\n  Exit code:    {rc}\n"
            "--------------------------------------------------------------------------\n")
        return rc if rc > 0 else 1
    return 0


def main():
    sys.exit(run(sys.argv[1:]))


if __name__ == "__main__":
    main()

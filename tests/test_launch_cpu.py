"""Launcher plumbing on CPU: chart -> release -> controllers -> replica processes.

Covers the env contracts of the training-operator (PET_* / MASTER_* / HOSTNAME), elastic
rendezvous env, OnFailure gang restarts within backoffLimit, the MPIJob mpirun emulation
(OMPI_COMM_WORLD_* env, --output-filename files, --tag-output), the Pod kind
(data-process), the KFP-style pipeline with the exit-code fix, and PVC path rewriting
(SURVEY §2.3, §2.4, §3.1-§3.6, §5.3).
"""
import json
import os
import subprocess
import sys
import time

import pytest
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHARTS = os.path.join(REPO, "charts", "machine-learning")


@pytest.fixture()
def home(tmp_path, monkeypatch):
    monkeypatch.setenv("MXTRAIN_HOME", str(tmp_path / "home"))
    monkeypatch.setenv("MXTRAIN_NUM_GPUS", "0")
    monkeypatch.setenv("MXTRAIN_PV_LINK", "0")   # never symlink /fsx on the test host
    return tmp_path


def _values(tmp_path, doc, name="v.yaml"):
    p = tmp_path / name
    p.write_text(yaml.safe_dump(doc))
    return str(p)


def _install(chart, rel_name, files, sets=(), timeout=120):
    from mxtrain.launch import release as rel
    return rel.install(os.path.join(CHARTS, chart), rel_name, value_files=files, sets=list(sets), wait=True,
                       timeout=timeout)


def _log(rel_name, pod):
    from mxtrain.launch import release as rel
    return rel.logs(rel_name, pod=pod)


ENV_PROBE = ("import os,json; print('ENV', json.dumps({k: os.environ.get(k) for k in "
             "['HOSTNAME','PET_NNODES','PET_NPROC_PER_NODE','PET_NODE_RANK','PET_MASTER_ADDR','PET_MASTER_PORT',"
             "'PET_RDZV_ENDPOINT','PET_RDZV_ID','PET_RDZV_BACKEND','HOME','WORLD_SIZE','RANK']}))")


def _env_from_log(text):
    for line in text.splitlines():
        if line.startswith("ENV "):
            return json.loads(line[4:])
    raise AssertionError(f"no ENV line in log:\n{text}")


def test_pytorchjob_distributed_env_contract(home):
    v = _values(home, {
        "resources": {"nnodes": 3, "nproc_per_node": 2},
        "pvc": [{"name": "pv-fsx", "mount_path": "/fsx"}, {"name": "pv-efs", "mount_path": "/efs"}],
        "train": {"env": [{"name": "HOME", "value": "/efs/home/{{ .Release.Name }}"}],
                  "command": ["python3"], "args": ["-c", f'"{ENV_PROBE}"']}})
    st = _install("training/pytorchjob-distributed", "envtest", [v])
    assert st["phase"] == "Succeeded", st
    pods = st["resources"]["PyTorchJob/pytorchjob-envtest"]["pods"]
    assert sorted(pods) == ["pytorchjob-envtest-master-0", "pytorchjob-envtest-worker-0", "pytorchjob-envtest-worker-1"]
    ports = set()
    for rank, pod in enumerate(sorted(pods)):
        log = _log("envtest", pod)
        assert "Training script done" in log
        env = _env_from_log(log)
        assert env["HOSTNAME"] == pod
        assert env["PET_NNODES"] == "3" and env["PET_NPROC_PER_NODE"] == "2"
        assert env["PET_NODE_RANK"] == str(rank)
        assert env["PET_MASTER_ADDR"] == "127.0.0.1"
        ports.add(env["PET_MASTER_PORT"])
        # /efs is prefix-rewritten to the local PV root, layout below it unchanged
        assert env["HOME"].endswith(os.path.join("pv", "pv-efs", "home", "envtest"))
    assert len(ports) == 1


def test_pytorchjob_elastic_env_contract(home):
    v = _values(home, {
        "resources": {"nnodes": 1, "nproc_per_node": 1},
        "elastic_policy": {"rdzv_backend": "c10d", "rdzv_port": 0, "min_replicas": 1, "max_replicas": 2},
        "train": {"command": ["python3"], "args": ["-c", f'"{ENV_PROBE}"']}})
    st = _install("training/pytorchjob-elastic", "el", [v])
    assert st["phase"] == "Succeeded", st
    env = _env_from_log(_log("el", "pytorchjob-el-worker-0"))
    assert env["PET_RDZV_ID"] == "el"
    assert env["PET_RDZV_BACKEND"] == "c10d"
    assert env["PET_RDZV_ENDPOINT"].startswith("127.0.0.1:")
    assert env["PET_NNODES"] == "1:2"


def test_gang_restart_within_backoff(home):
    marker = home / "attempts"
    cmd = (f"import os,sys; p='{marker}'; n=int(open(p).read()) if os.path.exists(p) else 0; "
           f"open(p,'w').write(str(n+1)); sys.exit(0 if n>=2 else 3)")
    v = _values(home, {"backoff_limit": 5, "resources": {"nnodes": 1},
                       "train": {"command": ["python3"], "args": ["-c", f'"{cmd}"']}})
    st = _install("training/pytorchjob-distributed", "rs", [v])
    assert st["phase"] == "Succeeded", st
    assert st["resources"]["PyTorchJob/pytorchjob-rs"]["restarts"] == 2
    # exhausted budget -> Failed
    marker.unlink()
    v = _values(home, {"backoff_limit": 1, "resources": {"nnodes": 1},
                       "train": {"command": ["python3"], "args": ["-c", f'"{cmd}"']}}, "v2.yaml")
    st = _install("training/pytorchjob-distributed", "rs2", [v])
    assert st["phase"] == "Failed"


def test_failure_masked_by_echo_like_reference(home):
    # the script contract: `cmd && echo done` is the last command -> exit status is the
    # training command's (no post_script), so a failing command fails the replica.
    v = _values(home, {"backoff_limit": 0, "resources": {"nnodes": 1},
                       "train": {"command": ["false"]}})
    st = _install("training/pytorchjob-distributed", "fail", [v])
    assert st["phase"] == "Failed"


def test_mpijob_ranks_and_output_files(home):
    probe = ("import os; print('RANK', os.environ['OMPI_COMM_WORLD_RANK'], os.environ['OMPI_COMM_WORLD_SIZE'], "
             "os.environ['OMPI_COMM_WORLD_LOCAL_RANK'], os.environ['HOSTNAME'], os.environ['HOME'])")
    v = _values(home, {
        "resources": {"gpu_nodes": 2, "gpus_per_node": 2, "gpu_instance_type": "mi355x.8x"},
        "train": {"command": ["python3"], "args": ["-c", f'"{probe}"']}})
    st = _install("training/mpijob-horovod-tensorflow-gpu", "mpi", [v])
    assert st["phase"] == "Succeeded", st
    log = _log("mpi", "mpijob-mpi-launcher")
    rows = sorted(line.split("RANK ", 1)[1].split() for line in log.splitlines() if "<stdout>:RANK " in line)
    assert [r[0] for r in rows] == ["0", "1", "2", "3"]
    assert all(r[1] == "4" for r in rows)
    assert [r[3] for r in rows] == ["mpijob-mpi-worker-0"] * 2 + ["mpijob-mpi-worker-1"] * 2
    assert [r[2] for r in rows] == ["0", "1", "0", "1"]
    assert "[1,0]<stdout>:" in log and "JOB MAP" in log
    home_dir = rows[0][4]
    outs = [d for d in os.listdir(os.path.join(home_dir, "logs")) if d.startswith("mpi-")]
    assert len(outs) == 1
    files = os.path.join(home_dir, "logs", outs[0], "1")
    assert sorted(os.listdir(files)) == ["rank.0", "rank.1", "rank.2", "rank.3"]
    assert "RANK 2" in open(os.path.join(files, "rank.2", "stdout")).read()


def test_mpirun_abort_on_rank_failure(tmp_path):
    script = tmp_path / "r.sh"
    script.write_text("#!/bin/bash\nif [ $OMPI_COMM_WORLD_RANK = 1 ]; then exit 7; fi\nsleep 30\n")
    script.chmod(0o755)
    env = dict(os.environ, MXTRAIN_MPI_SLOTS="3", PYTHONPATH=REPO)
    env.pop("MXTRAIN_MPI_WORKERS", None)
    r = subprocess.run([sys.executable, "-m", "mxtrain.launch.mpirun", "-np", "3", str(script)], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 7
    assert "Exit code:    7" in r.stderr


def test_data_process_pod(home):
    v = _values(home, {"pvc": [{"name": "pv-fsx", "mount_path": "/fsx"}],
                       "pre_script": ["mkdir -p /fsx/data/x", "echo hello > /fsx/data/x/f.txt"],
                       "process": {"command": ["cat"], "args": ["/fsx/data/x/f.txt"]}})
    st = _install("data-prep/data-process", "dp", [v])
    assert st["phase"] == "Succeeded", st
    log = _log("dp", "data-process-dp")
    assert "hello" in log and "Processing script done" in log
    assert (home / "home" / "pv" / "pv-fsx" / "data" / "x" / "f.txt").exists()


def test_pipeline_stops_on_failure_and_keeps_exit_code(home):
    from mxtrain.launch import release as rel
    from mxtrain.pipeline import run_pipeline
    ok = {"release_name": "p1", "namespace": "default", "path": "charts/machine-learning/data-prep/data-process",
          "values": {"process": {"command": ["true"]}}}
    bad = {"release_name": "p2", "namespace": "default", "path": "charts/machine-learning/data-prep/data-process",
           "values": {"process": {"command": ["false"]}}}
    never = dict(ok, release_name="p3")
    logs = []
    assert run_pipeline([ok, bad, never], log=logs.append) == "Failure"
    assert rel.read_status("p1", "default")["phase"] == "Uninstalled"
    assert rel.read_status("p2", "default")["phase"] == "Uninstalled"
    with pytest.raises(FileNotFoundError):
        rel.read_status("p3", "default")
    assert run_pipeline([ok], log=logs.append) == "Success"


def test_cli_install_status_uninstall(home):
    v = _values(home, {"resources": {"nnodes": 1}, "train": {"command": ["sleep"], "args": ["30"]}})
    env = dict(os.environ, PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-m", "mxtrain", "install", "bg",
                        os.path.join(CHARTS, "training/pytorchjob-distributed"), "-f", v],
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    from mxtrain.launch import release as rel
    import time
    t0 = time.time()
    while rel.read_status("bg")["phase"] != "Running" and time.time() - t0 < 30:
        time.sleep(0.2)
    assert rel.read_status("bg")["phase"] == "Running"
    pid = rel.read_status("bg")["resources"]["PyTorchJob/pytorchjob-bg"]["pods"]["pytorchjob-bg-master-0"]["pid"]
    r = subprocess.run([sys.executable, "-m", "mxtrain", "uninstall", "bg"], env=env, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    time.sleep(0.5)
    with pytest.raises(ProcessLookupError):
        os.kill(pid, 0)
    assert not os.path.exists(rel.release_dir("bg"))


def test_storage_rewrite_keeps_layout(tmp_path, monkeypatch):
    from mxtrain.runtime.storage import plan_mounts
    monkeypatch.setenv("MXTRAIN_PV_ROOT", str(tmp_path / "pv"))
    plan = plan_mounts([{"name": "pv-1", "mountPath": "/fsx"}],
                       [{"name": "pv-1", "persistentVolumeClaim": {"claimName": "pv-fsx"}}], allow_link=False)
    s = plan.rewrite("--save /fsx/home/r/checkpoints/0 --x /fsxother /a/fsx/b")
    assert s == f"--save {tmp_path}/pv/pv-fsx/home/r/checkpoints/0 --x /fsxother /a/fsx/b"


def test_gpu_ledger_disjoint(tmp_path):
    from mxtrain.runtime.topology import NodeLedger
    a = NodeLedger(str(tmp_path / "l.json"), "a", total=8)
    b = NodeLedger(str(tmp_path / "l.json"), "b", total=8)
    ga = a.allocate(4)
    gb = b.allocate(4)
    assert not set(ga) & set(gb)
    with pytest.raises(RuntimeError):
        b.allocate(1)
    a.release(ga)
    assert len(b.allocate(4)) == 4


def test_hpo_random_and_grid_search(home, tmp_path):
    """Katib-style experiment over the data-process chart: the trial prints a loss that
    is minimal at x=3; grid search must find it, StdOut collector parses it."""
    from mxtrain.hpo import run_experiment
    exp = {"name": "quad", "objective": {"type": "minimize", "objectiveMetricName": "loss"},
           "algorithm": {"algorithmName": "grid"}, "parallelTrialCount": 2, "maxTrialCount": 5,
           "parameters": [{"name": "x", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "5"}}],
           "trialTemplate": {"chart": os.path.join(CHARTS, "data-prep", "data-process"),
                             "set": ["process.command[0]=python3", "process.args[0]=-c",
                                     "process.args[1]=\"print('step 10 loss: %f' % ((${trialParameters.x}-3)**2+0.5))\""]}}
    res = run_experiment(exp, log=lambda *a: None)
    assert res["condition"] == "Succeeded" and len(res["trials"]) == 5
    assert res["best"]["parameters"]["x"] == "3" and res["best"]["metrics"]["loss"] == pytest.approx(0.5)
    exp["algorithm"] = {"algorithmName": "random", "seed": 1}
    exp["name"] = "quad-r"
    exp["earlyStopping"] = {"algorithmName": "medianstop", "minTrialsRequired": 2}
    res = run_experiment(exp, log=lambda *a: None)
    assert {t["status"] for t in res["trials"]} <= {"Succeeded", "EarlyStopped"}


# --------------------------------------------------------------------------- CPU / NUMA placement
def fake_topology(root, sockets=2, cores=32, smt=2, gpus_per_socket=4, io_link_only=()):
    """Fake sysfs: `sockets` NUMA nodes of `cores` SMT-`smt` cores (CPU numbering as on
    Linux: all first threads, then the siblings), KFD CPU nodes first, then the GPUs
    with PCI locations whose numa_node says their socket (GPUs in `io_link_only` carry
    only a KFD io_link to their CPU node)."""
    ncpu = sockets * cores
    for s in range(sockets):
        first = list(range(s * cores, (s + 1) * cores))
        cpus = first + [c + ncpu * t for t in range(1, smt) for c in first]
        d = root / f"sys/devices/system/node/node{s}"
        d.mkdir(parents=True)
        from mxtrain.runtime.affinity import format_cpulist
        (d / "cpulist").write_text(format_cpulist(cpus) + "\n")
        for c in first:
            sib = [c + ncpu * t for t in range(smt)]
            for x in sib:
                t = root / f"sys/devices/system/cpu/cpu{x}/topology"
                t.mkdir(parents=True, exist_ok=True)
                (t / "thread_siblings_list").write_text(",".join(map(str, sib)) + "\n")
    kfd = root / "sys/class/kfd/kfd/topology/nodes"
    for s in range(sockets):
        n = kfd / str(s)
        n.mkdir(parents=True)
        (n / "properties").write_text(f"cpu_cores_count {cores * smt}\nsimd_count 0\ngfx_target_version 0\n")
    for g in range(sockets * gpus_per_socket):
        s = g // gpus_per_socket
        n = kfd / str(sockets + g)
        (n / "io_links/0").mkdir(parents=True)
        (n / "io_links/0/properties").write_text(f"type 11\nnode_from {sockets + g}\nnode_to {s}\n")
        bus = 0x10 + 0x10 * g
        if g in io_link_only:
            (n / "properties").write_text("cpu_cores_count 0\nsimd_count 1024\ngfx_target_version 90500\n")
            continue
        (n / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\ngfx_target_version 90500\n"
                                      f"location_id {bus << 8}\ndomain 0\n")
        p = root / f"sys/bus/pci/devices/0000:{bus:02x}:00.0"
        p.mkdir(parents=True)
        (p / "numa_node").write_text(f"{s}\n")
    return root


def test_numa_plan_disjoint_local_8_ranks(tmp_path):
    from mxtrain.runtime import affinity as af
    root = str(fake_topology(tmp_path, io_link_only=(5,)))
    assert af.gpu_numa_nodes(root) == [0, 0, 0, 0, 1, 1, 1, 1]
    nodes = af.numa_cpus(root)
    allowed = range(128)
    pl = af.plan(list(range(8)), "core", root=root, allowed=allowed)
    seen = set()
    for p in pl:
        assert p.numa == p.gpu // 4
        assert set(p.cpus) <= set(nodes[p.numa])                  # NUMA-local
        assert not (set(p.cpus) & seen)                           # disjoint
        assert len(p.cpus) == 16                                  # 8 cores x 2 threads
        assert all((c + 64) in p.cpus for c in p.cpus if c < 64)  # SMT siblings kept together
        seen |= set(p.cpus)
    assert len(seen) == 128
    # a GPU subset + rank order from a launcher (HIP ids 6,1 -> numa 1, 0)
    pl = af.plan([6, 1], "core", root=root, allowed=allowed)
    assert [p.numa for p in pl] == [1, 0] and len(pl[0].cpus) == 64
    # numa/socket: whole local node; hwthread: a single CPU; bad mode raises
    assert af.plan([0, 7], "numa", root=root, allowed=allowed)[1].cpus == nodes[1]
    assert len(af.plan([0], "hwthread", root=root, allowed=allowed)[0].cpus) == 1
    with pytest.raises(ValueError):
        af.plan([0], "bogus", root=root)
    # cpuset restricted by the launcher's own affinity
    pl = af.plan([0, 1], "core", root=root, allowed=[0, 1, 2, 3, 64, 65, 66, 67])
    assert pl[0].cpus == [0, 1, 64, 65] and pl[1].cpus == [2, 3, 66, 67]
    # env round trip for torchrun-started local ranks
    env = af.rank_env(pl)
    assert af.parse_cpulist(json.loads(env["MXTRAIN_RANK_CPUSETS"])[1]) == [2, 3, 66, 67]


def _small_topology(tmp_path):
    # the test host may have only a few CPUs: 2 sockets x 2 cores x SMT2 over cpus 0-7
    n = min(8, len(os.sched_getaffinity(0)))
    assert n >= 8 or pytest.skip("needs 8 CPUs")
    return fake_topology(tmp_path / "sysfs", sockets=2, cores=2, smt=2, gpus_per_socket=2)


def test_mpirun_binds_ranks_numa_local(tmp_path):
    root = _small_topology(tmp_path)
    wf = tmp_path / "workers.json"
    wf.write_text(json.dumps({"workers": [{"name": "w0", "gpus": [0, 2]}, {"name": "w1", "gpus": [1, 3]}],
                              "slots": 2}))
    probe = ("import os, json; print('AFF', os.environ['OMPI_COMM_WORLD_RANK'], "
             "json.dumps(sorted(os.sched_getaffinity(0)), separators=(',', ':')))")
    env = dict(os.environ, PYTHONPATH=REPO, MXTRAIN_SYSFS_ROOT=str(root), MXTRAIN_MPI_WORKERS=str(wf),
               MXTRAIN_MPI_PLACEMENT=str(tmp_path / "pl.json"))
    r = subprocess.run([sys.executable, "-m", "mxtrain.launch.mpirun", "-np", "4", "-bind-to", "core",
                        "--report-bindings", "--tag-output", sys.executable, "-c", probe],
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    aff = {}
    for line in r.stdout.splitlines():
        if "AFF " in line:
            rank, lst = line.split("AFF ", 1)[1].split()
            aff[int(rank)] = json.loads(lst)
    # map-by slot: ranks 0,1 on w0 (GPUs 0,2 -> numa 0,1), ranks 2,3 on w1 (GPUs 1,3 -> numa 0,1)
    node0, node1 = {0, 1, 4, 5}, {2, 3, 6, 7}
    assert set(aff[0]) <= node0 and set(aff[2]) <= node0
    assert set(aff[1]) <= node1 and set(aff[3]) <= node1
    assert not set(aff[0]) & set(aff[2]) and not set(aff[1]) & set(aff[3])
    assert "MCW rank 3 bound to numa 1" in r.stderr
    pl = json.loads((tmp_path / "pl.json").read_text())
    assert pl["bind_to"] == "core" and [x["gpu"] for x in pl["ranks"]] == [0, 2, 1, 3]
    # -bind-to none (the reference's setting) leaves ranks unpinned
    r = subprocess.run([sys.executable, "-m", "mxtrain.launch.mpirun", "-np", "2", "-bind-to", "none",
                        sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    full = sorted(os.sched_getaffinity(0))
    rows = [line.split()[2] for line in r.stdout.splitlines() if line.startswith("AFF")]
    assert len(rows) == 2 and all(json.loads(x) == full for x in rows)


def test_pytorchjob_records_and_applies_placement(home, monkeypatch):
    root = _small_topology(home)
    monkeypatch.setenv("MXTRAIN_SYSFS_ROOT", str(root))
    monkeypatch.setenv("MXTRAIN_NUM_GPUS", "4")
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    # (every replica lingers after printing: the job succeeds with its master and the
    # controller then stops the workers, so on a loaded host a worker still starting its
    # interpreter could be stopped before its line)
    probe = ("import os, json, time; print('AFF', os.environ['HOSTNAME'], os.environ['MXTRAIN_RANK_CPUSETS'].replace(' ', ''), "
             "json.dumps(sorted(os.sched_getaffinity(0)), separators=(',', ':')), flush=True); time.sleep(8)")
    v = _values(home, {"resources": {"nnodes": 2, "nproc_per_node": 2},
                       "train": {"command": ["python3"], "args": ["-c", f'"{probe}"']}})
    st = _install("training/pytorchjob-distributed", "numa", [v])
    assert st["phase"] == "Succeeded", st
    job = st["resources"]["PyTorchJob/pytorchjob-numa"]
    ranks = job["placement"]["ranks"]
    from mxtrain.runtime.affinity import parse_cpulist
    assert [r["gpu"] for r in ranks] == [0, 1, 2, 3] and [r["numa"] for r in ranks] == [0, 0, 1, 1]
    sets = [set(parse_cpulist(r["cpus"])) for r in ranks]
    assert all(not (sets[i] & sets[j]) for i in range(4) for j in range(i))
    for pod in ("pytorchjob-numa-master-0", "pytorchjob-numa-worker-0"):
        # the job succeeds with its master (training-operator semantics): a worker can
        # still be starting its interpreter on a loaded host, so give its log time
        deadline = time.time() + 60
        while True:
            log = _log("numa", pod)
            lines = [x for x in log.splitlines() if x.startswith("AFF")]
            if lines or time.time() > deadline:
                break
            time.sleep(0.5)
        assert lines, f"{pod}: no AFF line in its log:\n{log[-2000:]}"
        line = lines[0]
        _, host, per_rank, aff = line.split()
        i = 0 if "master" in pod else 2
        assert set(json.loads(aff)) == sets[i] | sets[i + 1]          # replica = its ranks' union
        assert [set(parse_cpulist(x)) for x in json.loads(per_rank)] == sets[i:i + 2]
        assert job["pods"][pod]["cpus"]

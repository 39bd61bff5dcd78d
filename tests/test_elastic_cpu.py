"""Elastic PyTorchJob on CPU/gloo (reference
charts/machine-learning/training/pytorchjob-elastic/templates/train.yaml:59-64 and the
training-operator CRD's elasticPolicy.maxRestarts).

* a worker killed by MXTRAIN_FAULT makes torchrun's elastic agents re-rendezvous; the
  job re-forms, resumes from the last checkpoint and ends on the exact single-process
  trajectory, without the controller gang-restarting anything;
* membership moves between minReplicas and maxReplicas with `mxtrain scale`;
* a failed replica is restarted alone within backoffLimit; fewer than minReplicas alive
  fails the job.
"""
import json
import os
import sys
import threading
import time

import pytest
import torch
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHART = os.path.join(REPO, "charts", "machine-learning", "training", "pytorchjob-elastic")


@pytest.fixture()
def home(tmp_path, monkeypatch):
    monkeypatch.setenv("MXTRAIN_HOME", str(tmp_path / "home"))
    monkeypatch.setenv("MXTRAIN_NUM_GPUS", "0")
    monkeypatch.setenv("MXTRAIN_PV_LINK", "0")
    monkeypatch.setenv("MXTRAIN_CPU_BIND", "none")
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    return tmp_path


def _values(tmp_path, doc, name="v.yaml"):
    p = tmp_path / name
    p.write_text(yaml.safe_dump(doc))
    return str(p)


def _torchrun_job(tmp_path, steps, extra_env=(), sleep=0.0, nnodes=2, mn=2, mx=2, max_restarts=3):
    args = ["-m", "torch.distributed.run", "--nnodes", "$PET_NNODES", "--nproc_per_node", "$PET_NPROC_PER_NODE",
            "--rdzv_id", "$PET_RDZV_ID", "--rdzv_backend", "c10d", "--rdzv_endpoint", "$PET_RDZV_ENDPOINT",
            "-m", "mxtrain.workloads.elastic.train", "--ckpt-dir", str(tmp_path / "ckpt"), "--steps", str(steps),
            "--global-batch", "48", "--step-sleep", str(sleep), "--out", str(tmp_path / "out.json")]
    env = [{"name": "OMP_NUM_THREADS", "value": "1"}] + [{"name": k, "value": v} for k, v in extra_env]
    return {"backoff_limit": 2, "resources": {"nnodes": nnodes, "nproc_per_node": 1},
            "elastic_policy": {"rdzv_backend": "c10d", "rdzv_port": 0, "min_replicas": mn, "max_replicas": mx,
                               "max_restarts": max_restarts, "rdzv_conf": {"last_call_timeout": 1}},
            "train": {"env": env, "command": [sys.executable], "args": args}}


def _all_logs(name):
    from mxtrain.launch import release as rel
    return rel.logs(name)


def _reference(steps):
    from mxtrain.workloads.elastic.train import reference
    return reference(steps, 48, 0.05)


def test_elastic_worker_fault_reforms_and_resumes(home):
    from mxtrain.launch import release as rel
    once = home / "fault-fired"
    v = _values(home, _torchrun_job(home, 12, extra_env=[("MXTRAIN_FAULT", "1:5:exit"),
                                                          ("MXTRAIN_FAULT_ONCE_FILE", str(once))]))
    st = rel.install(CHART, "elf", value_files=[v], wait=True, timeout=240)
    log = _all_logs("elf")
    assert st["phase"] == "Succeeded", (st, log[-4000:])
    job = st["resources"]["PyTorchJob/pytorchjob-elf"]
    assert once.exists() and "injecting exit" in log
    # the agents re-formed the group (restart round >= 1, both ranks, resumed mid-run) ...
    rounds = [line for line in log.splitlines() if "[elastic] round" in line]
    resumed = [r for r in rounds if "restart=0" not in r]
    assert resumed and all("world=2" in r for r in resumed), rounds
    assert any(int(r.rsplit("resume_step=", 1)[1]) >= 5 for r in resumed), rounds
    # ... without the operator gang-restarting replicas
    assert job["restarts"] == 0 and all(p["restarts"] == 0 for p in job["pods"].values())
    assert job["elastic"]["minReplicas"] == 2 and job["elastic"]["removed"] == []
    out = json.loads((home / "out.json").read_text())
    assert torch.allclose(torch.tensor(out["w"], dtype=torch.float64), _reference(12), atol=1e-10)


def test_elastic_scale_between_min_and_max(home):
    from mxtrain.launch import release as rel
    v = _values(home, _torchrun_job(home, 60, sleep=0.15, nnodes=1, mn=1, mx=2))
    res = {}
    th = threading.Thread(target=lambda: res.update(st=rel.install(CHART, "els", value_files=[v], wait=True,
                                                                  timeout=300)))
    th.start()

    def wait_for(pred, what, limit=120):
        t0 = time.time()
        while time.time() - t0 < limit:
            try:
                log = _all_logs("els")
            except (OSError, FileNotFoundError):
                log = ""
            if pred(log):
                return log
            time.sleep(0.3)
        raise AssertionError(f"timed out waiting for {what}:\n{log[-3000:]}")

    wait_for(lambda t: "world=1 rank=0 resume_step=0" in t, "first round with one replica")
    rel.scale("els", 5)                       # clamped to maxReplicas=2
    wait_for(lambda t: "world=2 rank=1" in t, "second replica joining")
    rel.scale("els", 1)
    wait_for(lambda t: t.count("world=1 rank=0") >= 2, "survivor re-forming alone")
    th.join(timeout=300)
    st = res["st"]
    assert st["phase"] == "Succeeded", (st, _all_logs("els")[-4000:])
    job = st["resources"]["PyTorchJob/pytorchjob-els"]
    assert job["elastic"]["removed"] == ["pytorchjob-els-worker-1"]
    assert job["elastic"]["maxReplicas"] == 2
    out = json.loads((home / "out.json").read_text())
    assert out["world"] == 1
    assert torch.allclose(torch.tensor(out["w"], dtype=torch.float64), _reference(60), atol=1e-10)


def test_elastic_replica_restart_alone_and_min_replicas(home):
    from mxtrain.launch import release as rel
    marker = home / "attempts"
    # replica 1 fails once, replica 0 keeps running: only replica 1 is restarted
    cmd = (f"import os,sys,time; r=os.environ['PET_NODE_RANK']; p='{marker}'; "
           f"n=int(open(p).read()) if os.path.exists(p) else 0; "
           f"(open(p,'w').write(str(n+1)), sys.exit(3)) if r=='1' and n==0 else time.sleep(2.0 if r=='0' else 0.2)")
    doc = {"backoff_limit": 3, "resources": {"nnodes": 2},
           "elastic_policy": {"rdzv_backend": "c10d", "rdzv_port": 0, "min_replicas": 1, "max_replicas": 2},
           "train": {"command": [sys.executable], "args": ["-c", f'"{cmd}"']}}
    st = rel.install(CHART, "elr", value_files=[_values(home, doc)], wait=True, timeout=120)
    assert st["phase"] == "Succeeded", st
    job = st["resources"]["PyTorchJob/pytorchjob-elr"]
    assert job["restarts"] == 1
    assert job["pods"]["pytorchjob-elr-worker-1"]["restarts"] == 1
    assert job["pods"]["pytorchjob-elr-worker-0"]["restarts"] == 0
    # budget spent and fewer than minReplicas alive -> Failed
    doc = {"backoff_limit": 0, "resources": {"nnodes": 2},
           "elastic_policy": {"rdzv_backend": "c10d", "rdzv_port": 0, "min_replicas": 2, "max_replicas": 2},
           "train": {"command": [sys.executable],
                     "args": ["-c", "\"import os,sys,time; sys.exit(5) if os.environ['PET_NODE_RANK']=='1' else time.sleep(30)\""]}}
    t0 = time.time()
    st = rel.install(CHART, "elm", value_files=[_values(home, doc, "v2.yaml")], wait=True, timeout=120)
    assert st["phase"] == "Failed" and time.time() - t0 < 25
    assert "minReplicas=2" in st["resources"]["PyTorchJob/pytorchjob-elm"]["message"]

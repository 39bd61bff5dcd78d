"""ML-platform layer on CPU: TensorBoard event files (native CRC-32C), Profiles with GPU
quotas, PodDefault injection into launched replicas, the central dashboard API
(§5.5)."""
import base64
import json
import os
import threading
import urllib.request

import pytest
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHARTS = os.path.join(REPO, "charts", "machine-learning")


@pytest.fixture()
def home(tmp_path, monkeypatch):
    monkeypatch.setenv("MXTRAIN_HOME", str(tmp_path / "home"))
    monkeypatch.setenv("MXTRAIN_NUM_GPUS", "0")
    monkeypatch.setenv("MXTRAIN_PV_LINK", "0")
    return tmp_path


def test_tfevents_roundtrip_and_crc(tmp_path):
    from mxtrain.obs import tensorboard as tb
    assert tb._py_crc32c(b"123456789") == 0xE3069283           # CRC-32C check value
    data = os.urandom(3000)
    assert tb.masked_crc32c(data) == ((((tb._py_crc32c(data) >> 15) | (tb._py_crc32c(data) << 17))
                                       + 0xA282EAD8) & 0xFFFFFFFF)
    with tb.SummaryWriter(str(tmp_path / "run1")) as w:
        for s in range(5):
            w.add_scalars_flat({"lm loss": 10.0 - s, "lr": 1e-4 * s}, s)
    with tb.SummaryWriter(str(tmp_path / "run2")) as w:
        w.add_scalar("lm loss", 3.5, 7)
    sc = tb.read_scalars(str(tmp_path))
    assert [v for _, _, v in sc["run1/lm loss"]] == [10.0, 9.0, 8.0, 7.0, 6.0]
    assert sc["run2/lm loss"][0][0] == 7 and sc["run2/lm loss"][0][2] == 3.5
    # first record is the file_version event
    p = tb.event_files(str(tmp_path / "run2"))[0]
    first = next(tb.read_records(p))
    assert tb.decode_event(first)["file_version"] == "brain.Event:2"
    # corruption is detected
    raw = bytearray(open(p, "rb").read())
    raw[-6] ^= 0xFF
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        list(tb.read_records(p))


def test_profile_quota_blocks_gpu_allocation(home):
    from mxtrain.mlplatform import profiles as pr
    from mxtrain.runtime.topology import NodeLedger
    pr.create("team-a", owner="a@x", gpu_quota=2, contributors=["b@x"])
    assert pr.gpu_quota("team-a") == 2
    assert pr.can("a@x", "delete", "team-a") and pr.can("b@x", "create", "team-a")
    assert not pr.can("c@x", "get", "team-a") and not pr.can("b@x", "admin", "team-a")
    led_path = str(home / "home" / "gpu-ledger.json")
    l1 = NodeLedger(led_path, "team-a/job1", total=8)
    assert len(l1.allocate(2)) == 2
    l2 = NodeLedger(led_path, "team-a/job2", total=8)
    with pytest.raises(RuntimeError, match="exceeded quota"):
        l2.allocate(1)
    l3 = NodeLedger(led_path, "team-b/job", total=8)     # no profile -> no quota
    assert len(l3.allocate(4)) == 4


def test_pod_default_injected_into_replicas(home):
    from mxtrain.launch import release as rel
    from mxtrain.mlplatform import profiles as pr
    ns = "kubeflow-user-example-com"
    pr.load(ns)   # default profile with access-ml-pipeline
    pr.set_pod_default(ns, {"name": "hf-offline",
                            "selector": {"matchExpressions": [
                                {"key": "app.kubernetes.io/managed-by", "operator": "Exists"}]},
                            "env": [{"name": "HF_HUB_OFFLINE", "value": "1"},
                                    {"name": "HOME", "value": "/should/not/override"}]})
    v = home / "v.yaml"
    v.write_text(yaml.safe_dump({"train": {"env": [{"name": "HOME", "value": str(home / "h")}],
                                           "command": ["python3", "-c"],
                                           "args": ["\"import os; print('PD', os.environ.get('HF_HUB_OFFLINE'), "
                                                    "os.environ['HOME'], os.environ.get('MXTRAIN_POD_DEFAULTS'))\""]},
                                 "resources": {"nnodes": 1, "nproc_per_node": 1}}))
    st = rel.install(os.path.join(CHARTS, "training/pytorchjob-distributed"), "pdtest", value_files=[str(v)],
                     wait=True, timeout=120)
    assert st["phase"] == "Succeeded", st
    log = rel.logs("pdtest", ns, None)
    assert f"PD 1 {home / 'h'} hf-offline" in log, log


def test_dashboard_routes_and_auth(home, tmp_path):
    from mxtrain.launch import release as rel
    from mxtrain.mlplatform import dashboard as db
    from mxtrain.obs.tensorboard import SummaryWriter
    v = home / "v.yaml"
    v.write_text(yaml.safe_dump({"pvc": [{"name": "pv-fsx", "mount_path": "/fsx"}],
                                 "pre_script": ["mkdir -p /fsx/data", "echo hi > /fsx/data/a.txt"],
                                 "process": {"command": ["true"]}}))
    st = rel.install(os.path.join(CHARTS, "data-prep/data-process"), "dash", value_files=[str(v)],
                     wait=True, timeout=120)
    assert st["phase"] == "Succeeded"
    from mxtrain.runtime.storage import pv_root
    tbdir = os.path.join(pv_root(), "pv-fsx", "tb")
    with SummaryWriter(tbdir) as w:
        w.add_scalar("loss", 2.0, 1)
    with SummaryWriter(str(tmp_path / "outside")) as w:
        w.add_scalar("loss", 2.0, 1)
    code, _, body = db.route("/api/jobs", {})
    assert code == 200 and any(j["name"] == "dash" and j["phase"] == "Succeeded" for j in json.loads(body))
    code, _, body = db.route("/api/jobs/kubeflow-user-example-com/dash/logs", {})
    assert code == 200 and "Processing script done" in body
    code, _, body = db.route("/api/volumes", {})
    vols = {x["name"]: x for x in json.loads(body)}
    assert vols["pv-fsx"]["files"] >= 1
    code, _, body = db.route("/api/volumes/pv-fsx", {"path": "data"})
    assert [e["name"] for e in json.loads(body)["entries"]] == ["a.txt"]
    assert db.route("/api/volumes/pv-fsx", {"path": "../../.."})[0] == 403
    # encoded separators in the claim / namespace / name segments cannot escape
    assert db.route("/api/volumes/..%2F..%2F..", {"path": "etc"})[0] == 403
    assert db.route("/api/volumes/no-such-claim", {})[0] == 404
    assert db.route("/api/jobs/..%2F..%2F../dash/logs", {})[0] == 403
    assert db.route("/api/jobs/kubeflow-user-example-com/..%2Fx/logs", {})[0] == 403
    assert db.route("/api/jobs/kubeflow-user-example-com/..", {})[0] == 403
    assert db.route("/api/jobs/kubeflow-user-example-com/dash/logs", {"pod": "../x"})[0] == 403
    code, _, body = db.route("/api/tensorboards", {"logdir": tbdir})
    assert json.loads(body)["loss"][0]["value"] == 2.0
    assert db.route("/tensorboard", {"logdir": tbdir})[2].count("<svg") == 1
    assert db.route("/api/tensorboards", {"logdir": "pvc://pv-fsx/tb"})[0] == 200
    # the viewer reads only under the PV root / mxtrain home
    assert db.route("/api/tensorboards", {"logdir": str(tmp_path / "outside")})[0] == 403
    assert db.route("/tensorboard", {"logdir": "/etc"})[0] == 403
    assert db.route("/api/nope", {})[0] == 404
    for p in ("/", "/api", "/api/node", "/api/profiles", "/api/experiments", "/api/pipelines"):
        assert db.route(p, {})[0] == 200, p
    # live server with basic auth
    ht = tmp_path / "htpasswd"
    ht.write_text("admin:{SHA}" + base64.b64encode(__import__("hashlib").sha1(b"pw").digest()).decode() + "\n")
    srv = db.make_server("127.0.0.1", 0, db.Auth(str(ht)))
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}/api/jobs"
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(url, timeout=10)
        assert e.value.code == 401
        req = urllib.request.Request(url, headers={"Authorization": "Basic " + base64.b64encode(b"admin:pw").decode()})
        assert json.loads(urllib.request.urlopen(req, timeout=10).read())
    finally:
        srv.shutdown()


def test_node_init_stage_export_and_images(home, tmp_path, monkeypatch):
    import subprocess
    import sys
    repo_dir = tmp_path / "datarepo"
    (repo_dir / "coco").mkdir(parents=True)
    (repo_dir / "coco" / "a.json").write_text("{}")
    cfg = tmp_path / "node.yaml"
    base = yaml.safe_load(open(os.path.join(REPO, "infra", "node.yaml")))
    base["volumes"][1]["data_repository"] = {"import_path": str(repo_dir)}
    base["profiles"][0]["gpu_quota"] = 4
    cfg.write_text(yaml.safe_dump(base))
    env = dict(os.environ, PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-m", "mxtrain", "node", "init", "-f", str(cfg)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rep = json.loads(r.stdout)
    pv = home / "home" / "pv"
    assert rep["volumes"]["pv-fsx"]["import"]["copied"] == 1
    assert (pv / "pv-fsx" / "coco" / "a.json").exists() and (pv / "pv-efs" / "home").is_dir()
    from mxtrain.mlplatform import profiles as pr
    assert pr.gpu_quota("kubeflow-user-example-com") == 4
    src = tmp_path / "stage"
    src.mkdir()
    (src / "x.bin").write_bytes(b"1234")
    from mxtrain.tools import node_init as ni
    assert ni.stage_data(str(src), "pv-fsx:data/coco2017") == {"copied": 1, "skipped": 0}
    assert ni.stage_data(str(src), "pv-fsx:data/coco2017") == {"copied": 0, "skipped": 1}
    (pv / "pv-fsx" / "new.txt").write_text("n")
    assert ni.export_volume("pv-fsx")["copied"] >= 1 and (repo_dir / "new.txt").exists()
    assert {x["claim"] for x in ni.attach_info()} == {"pv-efs", "pv-fsx"}
    # image-reference rewriting of values files (build_and_push.sh)
    from mxtrain.tools import images
    vf = tmp_path / "vals" / "v.yaml"
    vf.parent.mkdir()
    vf.write_text("image: 'old/megatron:1'  # pinned\nx:\n  - image: other/img\n  image: \"{{ .Values.x }}\"\n")
    assert images.set_image("reg/mxtrain:rocm", [str(vf.parent)], match="megatron") == [str(vf)]
    txt = vf.read_text()
    assert "image: 'reg/mxtrain:rocm'  # pinned" in txt and "- image: other/img" in txt and "{{ .Values.x }}" in txt


def test_profile_and_debug_modes_reach_replicas(home, tmp_path):
    """mxtrain install --profile / --debug-mode: launch env in every replica, and the
    step profiler writes a trace + kernel table for its window."""
    import subprocess
    import sys
    v = home / "v.yaml"
    v.write_text(yaml.safe_dump({"train": {"env": [{"name": "HOME", "value": str(home / "h")}],
                                           "command": ["python3", "-c"],
                                           "args": ["\"import os; print('ENV', os.environ.get('MXTRAIN_PROFILE'), "
                                                    "os.environ.get('AMD_SERIALIZE_KERNEL'), "
                                                    "os.environ.get('MXTRAIN_CHECK_FINITE'))\""]},
                                 "resources": {"nnodes": 1, "nproc_per_node": 1}}))
    env = dict(os.environ, PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-m", "mxtrain", "install", "pm", os.path.join(CHARTS, "training",
                        "pytorchjob-distributed"), "-f", str(v), "--wait", "--profile", "--debug-mode"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    from mxtrain.launch import release as rel
    assert "ENV torch 3 1" in rel.logs("pm")
    from mxtrain.obs.profile import StepProfiler, check_finite
    import torch
    prof = StepProfiler(0, out_dir=str(tmp_path / "prof"), mode="torch", steps="1:3")
    x = torch.randn(64, 64)
    for it in range(1, 5):
        (x @ x).sum()
        prof.step(it)
    assert (tmp_path / "prof" / "trace-rank0.json").exists()
    assert "Self CPU" in (tmp_path / "prof" / "kernels-rank0.txt").read_text()
    with pytest.raises(FloatingPointError):
        check_finite(3, loss=torch.tensor(float("nan")))


def test_pipelines_api_defs_runs_terminate(home):
    """KFP backend (C46): stored pipeline definitions, asynchronous runs over the HTTP API,
    run status, terminate of a running step (its release is uninstalled)."""
    import time
    from mxtrain import pipeline as pl
    from mxtrain.launch import release as rel
    from mxtrain.mlplatform import dashboard as db
    dp = "charts/machine-learning/data-prep/data-process"
    ok = {"release_name": "api-a", "namespace": "default", "path": dp, "values": {"process": {"command": ["true"]}}}
    ok2 = dict(ok, release_name="api-b")
    code, _, body = db.route("/api/pipelines/defs", {}, "POST",
                             json.dumps({"name": "two-steps", "chart_configs": [ok, ok2]}).encode())
    assert code == 201 and json.loads(body)["steps"] == 2
    assert [d["name"] for d in json.loads(db.route("/api/pipelines/defs", {})[2])] == ["two-steps"]
    assert db.route("/api/pipelines/defs", {}, "POST", b"{\"name\": \"../x\", \"chart_configs\": []}")[0] == 403
    srv = db.make_server("127.0.0.1", 0, db.Auth(None))
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}"
        # a text/plain or form POST is refused before it reaches the API
        req = urllib.request.Request(url + "/api/runs", data=json.dumps({"pipeline": "two-steps", "name": "rx"}).encode(),
                                     method="POST", headers={"Content-Type": "text/plain"})
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(req, timeout=30)
        assert e.value.code == 415
        req = urllib.request.Request(url + "/api/runs", data=json.dumps({"pipeline": "two-steps", "name": "r1"}).encode(),
                                     method="POST", headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=30) as r:
            assert r.status == 201 and json.loads(r.read())["run"] == "r1"
        rec = pl.wait_run("r1", timeout=120)
        assert rec["status"] == "Succeeded" and rec["result"] == "Success" and len(rec["steps"]) == 2
        with urllib.request.urlopen(url + "/api/runs/r1", timeout=30) as r:
            assert json.loads(r.read())["pipeline"] == "two-steps"
    finally:
        srv.shutdown()
    slow = dict(ok, release_name="api-slow", values={"process": {"command": ["sleep"], "args": ["60"]}})
    code, _, body = db.route("/api/runs", {}, "POST", json.dumps({"chart_configs": [slow, ok], "name": "r2"}).encode())
    assert code == 201
    t0 = time.time()
    while time.time() - t0 < 60:
        try:
            if rel.read_status("api-slow", "default")["phase"] == "Running":
                break
        except FileNotFoundError:
            pass
        time.sleep(0.2)
    # a user without a role in the run's namespace cannot terminate it
    assert db.route("/api/runs/r2/terminate", {}, "POST", user="mallory@example.com")[0] == 403
    code, _, body = db.route("/api/runs/r2/terminate", {}, "POST")
    assert code == 200 and json.loads(body)["terminating"]
    rec = pl.wait_run("r2", timeout=60)
    assert rec["status"] == "Terminated" and rec["result"] == "Failure" and len(rec["steps"]) == 1
    assert rel.read_status("api-slow", "default")["phase"] == "Uninstalled"
    assert time.time() - t0 < 45


def test_tensorboard_resources_runs_and_smoothing(home, tmp_path):
    """Tensorboards (C44): Tensorboard resources with pvc:// logspaths, one chart per tag
    with the runs overlaid, TensorBoard's debiased EMA smoothing, tag filter."""
    from mxtrain.mlplatform import dashboard as db
    from mxtrain.obs.tensorboard import SummaryWriter
    from mxtrain.runtime.storage import pv_root
    logs = os.path.join(pv_root(), "pv-fsx", "exp1")
    for run, scale in (("run-a", 1.0), ("run-b", 2.0)):
        with SummaryWriter(os.path.join(logs, run)) as w:
            for s in range(5):
                w.add_scalar("loss", scale / (s + 1), s)
                w.add_scalar("lr", 0.1, s)
    code, _, body = db.route("/api/tensorboards", {}, "POST",
                             json.dumps({"name": "tb1", "logspath": "pvc://pv-fsx/exp1"}).encode())
    assert code == 201 and json.loads(body)["url"] == "/tensorboard/tb1"
    assert db.route("/api/tensorboards", {}, "POST",
                    json.dumps({"name": "tb2", "logspath": "pvc://pv-fsx/../../etc"}).encode())[0] == 403
    # only pvc:// logspaths, and only in a namespace the user may write to
    assert db.route("/api/tensorboards", {}, "POST",
                    json.dumps({"name": "tb3", "logspath": "/etc"}).encode())[0] == 403
    assert db.route("/api/tensorboards", {}, "POST", json.dumps({"name": "tb4", "logspath": "pvc://pv-fsx/exp1"}).encode(),
                    user="mallory@example.com")[0] == 403
    assert [t["name"] for t in json.loads(db.route("/api/tensorboards", {})[2])] == ["tb1"]
    view = json.loads(db.route("/api/tensorboards", {"logdir": logs, "view": "tags"})[2])
    assert set(view) == {"loss", "lr"} and set(view["loss"]) == {"run-a", "run-b"}
    assert [p["value"] for p in view["loss"]["run-b"]][:2] == [2.0, 1.0]
    code, ctype, page = db.route("/tensorboard/tb1", {"tag": "^loss$", "smoothing": "0.5"})
    assert code == 200 and "run-a" in page and "run-b" in page and "<h3>loss</h3>" in page and "<h3>lr</h3>" not in page
    sm = db.smooth_ema([1.0, 0.0, 0.0], 0.5)
    assert sm[0] == 1.0 and abs(sm[1] - (0.5 * 0.5) / (1 - 0.25)) < 1e-12


def test_identity_tokens_and_node_certificates(home, tmp_path):
    """Dex + oauth2-proxy + cert-manager roles (C38-C40): password-grant JWTs accepted as
    bearer / session cookie, tampered / expired tokens refused, discovery + userinfo; node
    CA issuing a server certificate with SANs (renewal only near expiry) served over TLS."""
    import ssl
    import subprocess
    import urllib.error
    from mxtrain.mlplatform import dashboard as db
    from mxtrain.mlplatform import identity as idp
    idp.add_user("alice@example.com", "s3cret", ["ml"])
    assert idp.password_grant("alice@example.com", "s3cret")["token_type"] == "Bearer"
    with pytest.raises(PermissionError):
        idp.password_grant("alice@example.com", "wrong")
    tok = idp.issue_token("alice@example.com", 60)
    assert idp.verify_token(tok)["email"] == "alice@example.com"
    h, b, s = tok.split(".")
    with pytest.raises(PermissionError):
        idp.verify_token(f"{h}.{b}.{s[:-2]}AA")
    with pytest.raises(PermissionError):
        idp.verify_token(idp.issue_token("alice@example.com", -5))
    c = idp.issue_cert("dash", ["localhost"], ["127.0.0.1"])
    assert c["renewed"] == "yes" and idp.issue_cert("dash", ["localhost"], ["127.0.0.1"])["renewed"] == "no"
    r = subprocess.run(["openssl", "verify", "-CAfile", c["ca"], c["cert"]], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    txt = subprocess.run(["openssl", "x509", "-in", c["cert"], "-noout", "-text"], capture_output=True, text=True).stdout
    assert "DNS:localhost" in txt and "IP Address:127.0.0.1" in txt
    srv = db.make_server("127.0.0.1", 0, db.Auth(None, oidc=True), c["cert"], c["key"])
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    ctx = ssl.create_default_context(cafile=c["ca"])
    url = f"https://localhost:{srv.server_address[1]}"
    try:
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(url + "/api", context=ctx, timeout=30)
        assert e.value.code == 401
        with urllib.request.urlopen(url + "/.well-known/openid-configuration", context=ctx, timeout=30) as r:
            assert json.loads(r.read())["token_endpoint"].endswith("/auth/token")
        req = urllib.request.Request(url + "/auth/token", data=b"username=alice%40example.com&password=s3cret",
                                     headers={"Content-Type": "application/x-www-form-urlencoded"}, method="POST")
        with urllib.request.urlopen(req, context=ctx, timeout=30) as r:
            cookie = r.headers["Set-Cookie"].split(";")[0]
            access = json.loads(r.read())["access_token"]
        for hdr in ({"Authorization": f"Bearer {access}"}, {"Cookie": cookie}):
            with urllib.request.urlopen(urllib.request.Request(url + "/api", headers=hdr), context=ctx, timeout=30) as r:
                assert r.status == 200
        with urllib.request.urlopen(urllib.request.Request(url + "/auth/userinfo",
                                                           headers={"Authorization": f"Bearer {access}"}),
                                    context=ctx, timeout=30) as r:
            assert json.loads(r.read()) == {"sub": "alice@example.com", "email": "alice@example.com", "groups": ["ml"]}
        bad = urllib.request.Request(url + "/auth/token", data=b"username=alice%40example.com&password=x",
                                     headers={"Content-Type": "application/x-www-form-urlencoded"}, method="POST")
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(bad, context=ctx, timeout=30)
        assert e.value.code == 401
    finally:
        srv.shutdown()


def test_platform_up_dry_run(home):
    """`mxtrain platform up` (the reference's Kubeflow module): profile + identity user +
    dashboard certificate in one step; idempotent on a second run."""
    import subprocess
    import sys
    env = dict(os.environ, PYTHONPATH=REPO, MXTRAIN_PLATFORM_PASSWORD="pw1")
    cmd = [sys.executable, "-m", "mxtrain", "platform", "up", "--user", "bob@example.com", "--namespace", "team-a",
           "--gpu-quota", "4", "--dry-run"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout)
    assert plan["profile_created"] and plan["user_created"] and plan["url"].startswith("https://")
    from mxtrain.mlplatform import identity as idp
    from mxtrain.mlplatform import profiles as pr
    assert idp.password_grant("bob@example.com", "pw1")["token_type"] == "Bearer"
    assert pr.gpu_quota("team-a") == 4 and pr.can("bob@example.com", "create", "team-a")
    r = subprocess.run(cmd, env=dict(env, MXTRAIN_PLATFORM_PASSWORD=""), capture_output=True, text=True, timeout=120,
                       stdin=subprocess.DEVNULL)
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout)
    assert "profile_created" not in plan and "user_created" not in plan


def test_pipelines_api_enforces_profile_roles(home):
    """An authenticated user may start pipeline runs only in namespaces whose profile lists
    them (owner / contributor); unauthenticated loopback use is unchanged."""
    from mxtrain.mlplatform import dashboard as db
    from mxtrain.mlplatform import profiles as pr
    pr.create("team-b", owner="carol@example.com")
    cfg = {"release_name": "rb", "namespace": "team-b", "path": "charts/machine-learning/data-prep/data-process",
           "values": {"process": {"command": ["true"]}}}
    body = json.dumps({"name": "p-b", "chart_configs": [cfg]}).encode()
    assert db.route("/api/pipelines/defs", {}, "POST", body, user="mallory@example.com")[0] == 403
    assert db.route("/api/pipelines/defs", {}, "POST", body, user="carol@example.com")[0] == 201
    run = json.dumps({"pipeline": "p-b", "name": "rb1"}).encode()
    assert db.route("/api/runs", {}, "POST", run, user="mallory@example.com")[0] == 403


def test_pipeline_step_cache(home):
    """KFP cache server (C46): with caching on, a step whose chart files + values already
    succeeded is served from the cache (recorded with the execution it reused); a changed
    value, a failed step or a stale entry runs again."""
    from mxtrain import pipeline as pl
    from mxtrain.mlplatform import dashboard as db
    dp = "charts/machine-learning/data-prep/data-process"
    marker = home / "ran.txt"
    step = {"release_name": "c-a", "namespace": "default", "path": dp,
            "values": {"process": {"command": ["echo"], "args": ["x", ">>", str(marker)]}}}
    assert pl.run_pipeline([step], run_name="c1", cache=True) == "Success"
    assert pl.run_pipeline([step], run_name="c2", cache=True) == "Success"
    assert marker.read_text().count("x") == 1                      # second run: cached
    r2 = pl.get_run("c2")
    assert r2["steps"][0]["cached"] and r2["steps"][0]["cached_from"] == "c1"
    assert r2["steps"][0]["cache_key"] == pl.get_run("c1")["steps"][0]["cache_key"]
    # cache off (the default): runs again
    assert pl.run_pipeline([step], run_name="c3") == "Success"
    assert marker.read_text().count("x") == 2
    # a different value is a different key
    step2 = dict(step, values={"process": {"command": ["echo"], "args": ["y", ">>", str(marker)]}})
    assert pl.run_pipeline([step2], run_name="c4", cache=True) == "Success"
    assert "y" in marker.read_text() and not pl.get_run("c4")["steps"][0]["cached"]
    # staleness bound: an entry older than max_cache_staleness is not reused
    assert pl.run_pipeline([dict(step, max_cache_staleness=0)], run_name="c5", cache=True) == "Success"
    assert marker.read_text().count("x") == 3
    # failures are never cached
    bad = dict(step, release_name="c-bad", values={"process": {"command": ["false"]}})
    assert pl.run_pipeline([bad], run_name="c6", cache=True) == "Failure"
    assert pl.run_pipeline([bad], run_name="c7", cache=True) == "Failure"
    assert not pl.get_run("c7")["steps"][0]["cached"]
    # over the API: POST /api/runs {cache: true}
    code, _, body = db.route("/api/runs", {}, "POST", json.dumps({"chart_configs": [step], "name": "c8",
                                                                   "cache": True}).encode())
    assert code == 201
    rec = pl.wait_run("c8", timeout=60)
    assert rec["cache"] and rec["steps"][0]["cached"]


def test_pipeline_run_metadata_lineage(home):
    """KFP metadata store (MLMD, C46; mxtrain/mlmd.py): a run records a run context under its
    pipeline context, one execution per step with its Chart / ChartValues inputs and a
    ReleaseRecord output; a cached step is a CACHED execution pointing at (and outputting)
    what the producing execution wrote; a failed step is FAILED; artifact lineage walks back
    from an output to the producing execution and its inputs; served over the API."""
    from mxtrain import mlmd
    from mxtrain import pipeline as pl
    from mxtrain.mlplatform import dashboard as db
    dp = "charts/machine-learning/data-prep/data-process"
    step = {"release_name": "m-a", "namespace": "default", "path": dp,
            "values": {"process": {"command": ["echo"], "args": ["ok"]}}}
    bad = {"release_name": "m-b", "namespace": "default", "path": dp,
           "values": {"process": {"command": ["false"]}}}
    assert pl.run_pipeline([step], run_name="m1", pipeline="pm", cache=True) == "Success"
    assert pl.run_pipeline([step, bad], run_name="m2", pipeline="pm", cache=True) == "Failure"
    l1, l2 = mlmd.run_lineage("m1"), mlmd.run_lineage("m2")
    assert l1["run"]["parents"] == [{"type": "pipeline", "name": "pm"}]
    (e1,) = l1["executions"]
    assert e1["state"] == "COMPLETE" and e1["properties"]["exit_code"] == 0
    assert sorted(a["type"] for a in e1["inputs"]) == ["Chart", "ChartValues"]
    (out1,) = e1["outputs"]
    assert out1["type"] == "ReleaseRecord"
    c, f = l2["executions"]
    assert c["state"] == "CACHED" and c["properties"]["cached_from_run"] == "m1"
    assert c["properties"]["cached_from_execution"] == e1["id"]
    assert [a["id"] for a in c["outputs"]] == [out1["id"]]          # the reused output
    # identical inputs are shared artifacts
    assert sorted(a["id"] for a in c["inputs"]) == sorted(a["id"] for a in e1["inputs"])
    assert f["state"] == "FAILED" and f["properties"]["exit_code"] != 0
    assert pl.get_run("m2")["steps"][0]["execution_id"] == c["id"]
    lin = mlmd.artifact_lineage(out1["id"])
    assert lin["produced_by"] == [e1["id"], c["id"]]                # the producer and the cache hit
    assert lin["upstream"][0]["id"] == e1["id"] and len(lin["upstream"][0]["inputs"]) == 2
    code, _, body = db.route("/api/runs/m2/lineage", {})
    assert code == 200 and [e["state"] for e in json.loads(body)["executions"]] == ["CACHED", "FAILED"]
    code, _, body = db.route(f"/api/artifacts/{out1['id']}/lineage", {})
    assert code == 200 and json.loads(body)["artifact"]["type"] == "ReleaseRecord"
    assert db.route("/api/runs/nope/lineage", {})[0] == 404


def test_cron_expressions():
    import datetime as dt
    from mxtrain.pipeline import Cron
    t0 = dt.datetime(2026, 10, 17, 10, 7, 30).timestamp()           # a Saturday
    nxt = lambda e, t=t0: dt.datetime.fromtimestamp(Cron(e).next_after(t))  # noqa: E731
    assert nxt("*/15 * * * *") == dt.datetime(2026, 10, 17, 10, 15)
    assert nxt("0 2 * * 1-5") == dt.datetime(2026, 10, 19, 2, 0)         # next weekday
    assert nxt("0 0 1 * *") == dt.datetime(2026, 11, 1)
    assert nxt("30 0 9 * * 0") == dt.datetime(2026, 10, 18, 9, 0, 30)     # 6 fields (KFP): Sunday
    assert nxt("0 9 * * 7") == dt.datetime(2026, 10, 18, 9, 0)            # 7 = Sunday too
    assert nxt("0 12 29 2 *") == dt.datetime(2028, 2, 29, 12, 0)          # leap day
    for bad in ("* * *", "61 * * * *", "*/0 * * * *"):
        with pytest.raises(ValueError):
            Cron(bad)


def test_recurring_runs_schedule_concurrency_and_api(home):
    """ScheduledWorkflow (C46): interval / cron recurring runs of a stored pipeline, fired by
    Scheduler.tick, at most max_concurrency at once, no catch-up, enable / disable and
    end time; exposed under /api/recurringruns with KFAM checks."""
    import time
    from mxtrain import pipeline as pl
    from mxtrain.mlplatform import dashboard as db
    from mxtrain.mlplatform import profiles as pr
    dp = "charts/machine-learning/data-prep/data-process"
    ok = {"release_name": "rr-a", "namespace": "default", "path": dp, "values": {"process": {"command": ["true"]}}}
    pl.save_pipeline("nightly", [ok])
    submitted = []
    sch = pl.Scheduler(submit=lambda **kw: submitted.append(kw))
    code, _, body = db.route("/api/recurringruns", {}, "POST", json.dumps(
        {"name": "every-min", "pipeline": "nightly", "interval": 60, "cache": True}).encode())
    assert code == 201, body
    d = pl.get_recurring_run("every-min")
    t = d["created"]
    assert sch.tick(t + 30) == []                          # not due yet
    fired = sch.tick(t + 61)
    assert len(fired) == 1 and submitted[-1]["pipeline"] == "nightly" and submitted[-1]["cache"]
    assert submitted[-1]["recurring"] == "every-min"
    assert sch.tick(t + 62) == []                          # next period counts from the fire
    # no catch-up: a long gap fires once, not once per missed period
    assert len(sch.tick(t + 1000)) == 1 and sch.tick(t + 1001) == []
    # concurrency: a still-active run blocks the next period
    pl.save_pipeline("slow", [dict(ok, release_name="rr-slow", values={"process": {"command": ["sleep"],
                                                                                   "args": ["30"]}})])
    pl.save_recurring_run("slow-rr", "slow", interval=1, max_concurrency=1)
    real = pl.Scheduler()
    t1 = time.time() + 2
    assert len(real.tick(t1)) == 1
    assert real.tick(t1 + 5) == []                         # first run still active
    run = pl.get_recurring_run("slow-rr")["runs"][0]
    pl.terminate_run(run)
    pl.wait_run(run, timeout=60)
    assert pl.get_run(run)["recurring_run"] == "slow-rr"
    # the blocked period was SKIPPED, not delayed: the next fire is a period after the skip
    assert pl.get_recurring_run("slow-rr")["skipped"] == 1
    assert real.tick(t1 + 5.5) == []
    assert len(real.tick(t1 + 10)) == 1                    # free again
    for r in pl.get_recurring_run("slow-rr")["runs"]:
        pl.terminate_run(r)
        pl.wait_run(r, timeout=60)
    # disable / enable over the API; a user without a role in the namespace is refused
    pr.create("default", owner="owner@x")
    assert db.route("/api/recurringruns/every-min/disable", {}, "POST", user="mallory@x")[0] == 403
    assert db.route("/api/recurringruns/every-min/disable", {}, "POST", user="owner@x")[0] == 200
    assert sch.tick(time.time() + 10 ** 6) == [] or all("every-min" not in f for f in sch.tick(time.time() + 10 ** 6))
    assert json.loads(db.route("/api/recurringruns/every-min", {})[2])["next_fire"] is None
    assert db.route("/api/recurringruns/every-min/enable", {}, "POST")[0] == 200
    lst = json.loads(db.route("/api/recurringruns", {})[2])
    assert {x["name"] for x in lst} == {"every-min", "slow-rr"}
    # end time: nothing fires after it
    pl.save_recurring_run("ended", "nightly", cron="* * * * *", end_time=time.time() - 1)
    assert pl.next_fire(pl.get_recurring_run("ended")) is None
    # validation
    assert db.route("/api/recurringruns", {}, "POST", json.dumps(
        {"name": "bad", "pipeline": "nightly", "cron": "* * *"}).encode())[0] == 400
    assert db.route("/api/recurringruns", {}, "POST", json.dumps(
        {"name": "bad", "pipeline": "nightly"}).encode())[0] == 400
    assert db.route("/api/recurringruns", {}, "POST", json.dumps(
        {"name": "bad", "pipeline": "missing", "interval": 5}).encode())[0] == 404

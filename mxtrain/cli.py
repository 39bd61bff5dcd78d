"""`mxtrain` command line -- the helm/kubectl surface of the reference, single node
(README.md of the reference: `helm install --debug <rel> <chart> -f <values>`,
`kubectl logs -f`, `helm uninstall`).

    python -m mxtrain install <release> <chart> [-f values.yaml]... [--set k=v]... [--namespace ns] [--wait]
    python -m mxtrain uninstall <release> [--namespace ns]
    python -m mxtrain status <release> | list | logs <release> [--pod P] [-f]
    python -m mxtrain template <release> <chart> [-f ...] [--set ...]     (render only, helm template)
    python -m mxtrain lint <chart> [-f ...]
    python -m mxtrain pipeline run <pipeline.yaml>                        (KFP chart pipeline)
    python -m mxtrain node [--check]                                      (topology / GPU ledger / acceptance)
    python -m mxtrain node init -f infra/node.yaml | stage-data <src> <claim>:<path> | export <claim> | attach-pvc
    python -m mxtrain hpo run <experiment.yaml>                           (Katib-style search)
    python -m mxtrain dashboard [--port 8080]                             (central dashboard)
    python -m mxtrain profile create|list|delete|poddefault <ns> ...      (Profiles / PodDefaults)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

from .launch import release as rel


def _add_values(p):
    p.add_argument("-f", "--values", action="append", default=[], help="values YAML file (repeatable)")
    p.add_argument("--set", action="append", default=[], help="k=v override (repeatable)")
    p.add_argument("--set-string", action="append", default=[])
    p.add_argument("-n", "--namespace", default=rel.DEFAULT_NS)


def cmd_install(a):
    from .obs.profile import debug_env, profile_env
    launch_env = {}
    if a.profile:
        launch_env.update(profile_env("torch", a.profile_steps))
    if a.debug_mode:
        launch_env.update(debug_env())
    st = rel.install(a.chart, a.release, a.namespace, a.values, a.set, a.set_string, wait=a.wait,
                     timeout=a.timeout, launch_env=launch_env or None)
    if a.debug:
        print(open(os.path.join(rel.release_dir(a.release, a.namespace), "manifest.yaml")).read())
    print(f"NAME: {a.release}\nNAMESPACE: {a.namespace}\nSTATUS: {st.get('phase')}")
    if a.wait:
        _print_resources(st)
        return 0 if st.get("phase") == "Succeeded" else 1
    return 0


def _print_resources(st):
    for rname, r in (st.get("resources") or {}).items():
        print(f"  {rname}: {r.get('phase')} (restarts {r.get('restarts', 0)}) {r.get('message', '')}")
        for pname, p in (r.get("pods") or {}).items():
            print(f"    pod {pname}: {p.get('phase')} exit={p.get('exit_code')} gpus={p.get('gpus')}")


def cmd_uninstall(a):
    rel.uninstall(a.release, a.namespace)
    print(f'release "{a.release}" uninstalled')
    return 0


def cmd_scale(a):
    """Elastic PyTorchJob membership (kubectl scale analogue): the controller clamps to
    [minReplicas, maxReplicas]; new replicas join at the next rendezvous round."""
    rel.scale(a.release, a.replicas, a.namespace)
    print(f'release "{a.release}" scaled to {a.replicas} replica(s)')
    return 0


def cmd_status(a):
    st = rel.read_status(a.release, a.namespace)
    if a.output == "json":
        print(json.dumps(st, indent=1))
    else:
        print(f"NAME: {st['name']}\nNAMESPACE: {st['namespace']}\nSTATUS: {st.get('phase')}\n"
              f"MESSAGE: {st.get('message', '')}")
        _print_resources(st)
    return 0


def cmd_list(a):
    rows = rel.list_releases(a.namespace if not a.all_namespaces else None)
    print(f"{'NAME':24s} {'NAMESPACE':28s} {'STATUS':12s} CHART")
    for st in rows:
        print(f"{st['name']:24s} {st['namespace']:28s} {st.get('phase', ''):12s} {st.get('chart', '')}")
    return 0


def cmd_logs(a):
    if not a.follow:
        sys.stdout.write(rel.logs(a.release, a.namespace, a.pod))
        return 0
    d = os.path.join(rel.release_dir(a.release, a.namespace), "logs")
    offsets = {}
    while True:
        if os.path.isdir(d):
            for fn in sorted(os.listdir(d)):
                if a.pod and not fn.startswith(a.pod):
                    continue
                p = os.path.join(d, fn)
                with open(p, errors="replace") as f:
                    f.seek(offsets.get(fn, 0))
                    chunk = f.read()
                    offsets[fn] = f.tell()
                if chunk:
                    sys.stdout.write(chunk)
                    sys.stdout.flush()
        try:
            if rel.read_status(a.release, a.namespace).get("phase") in ("Succeeded", "Failed", "Terminated"):
                return 0
        except FileNotFoundError:
            return 0
        time.sleep(0.5)


def cmd_template(a):
    from .chart.render import load_chart, render_chart
    r = render_chart(load_chart(a.chart), a.release, a.namespace, a.values, a.set, a.set_string)
    sys.stdout.write(r.text)
    return 0


def cmd_lint(a):
    from .chart.lint import lint_chart
    problems = lint_chart(a.chart, a.values, a.set)
    for p in problems:
        print(p)
    failed = any(p.startswith("[ERROR]") for p in problems)
    print(f"1 chart(s) linted, {int(failed)} chart(s) failed")
    return 1 if failed else 0


def cmd_pipeline(a):
    from .pipeline import load_pipeline, run_pipeline
    res = run_pipeline(load_pipeline(a.file))
    print(res)
    return 0 if res == "Success" else 1


def cmd_hpo(a):
    from .hpo import load_experiment, run_experiment
    res = run_experiment(load_experiment(a.file), a.namespace)
    b = res["best"]
    print(json.dumps({"condition": res["condition"], "best": b and {"trial": b["trial"], "parameters": b["parameters"],
                                                                  "metrics": b["metrics"]}}, indent=1))
    return 0 if res["condition"] == "Succeeded" else 1


def cmd_node(a):
    from .tools import node_init as ni
    if a.action == "init":
        print(json.dumps(ni.init_node(ni.load_config(a.file)), indent=1))
        return 0
    if a.action == "stage-data":
        print(json.dumps(ni.stage_data(a.args[0], a.args[1])))
        return 0
    if a.action == "export":
        print(json.dumps(ni.export_volume(a.args[0])))
        return 0
    if a.action == "attach-pvc":
        print(json.dumps(ni.attach_info(), indent=1))
        return 0
    if a.check:
        from .runtime.nodecheck import main as nodecheck
        return nodecheck([] if a.gpus is None else ["--gpus", str(a.gpus)])
    from .runtime.topology import NODE_PROFILES, num_gpus
    from .runtime.storage import mxtrain_home, pv_root
    led = os.path.join(mxtrain_home(), "gpu-ledger.json")
    print(json.dumps({"gpus": num_gpus(), "profile": f"mi355x.{num_gpus()}x", "pv_root": pv_root(),
                      "ledger": json.load(open(led)) if os.path.exists(led) else {},
                      "profiles": NODE_PROFILES}, indent=1))
    return 0


def cmd_dashboard(a):
    from .mlplatform.dashboard import main as dash
    argv = ["--host", a.host, "--port", str(a.port)]
    for k in ("certfile", "keyfile", "htpasswd"):
        if getattr(a, k):
            argv += [f"--{k}", getattr(a, k)]
    for k in ("oidc", "tls_auto"):
        if getattr(a, k, False):
            argv.append("--" + k.replace("_", "-"))
    return dash(argv)


def cmd_identity(a):
    from .mlplatform.identity import main as idm
    return idm(a.args)


def cmd_platform(a):
    """The Kubeflow module of the reference (terraform kubeflow/): bring up the node's
    platform services in one step -- the user's profile (namespace, owner, GPU quota), the
    identity-provider user, the dashboard's certificate from the node CA, then the central
    dashboard behind TLS + OIDC sessions (jobs, volumes, tensorboards, HPO, pipelines API)."""
    from .mlplatform import identity as idp
    from .mlplatform import profiles as pr
    ns = a.namespace
    plan = {"profile": ns, "owner": a.user}
    if not any((p.get("metadata") or {}).get("name") == ns for p in pr.list_profiles()):
        pr.create(ns, owner=a.user, gpu_quota=a.gpu_quota)
        plan["profile_created"] = True
    if a.user not in idp.load_users():
        pw = os.environ.get("MXTRAIN_PLATFORM_PASSWORD") or sys.stdin.readline().rstrip("\n")
        if not pw:
            print("platform up: the first run needs the user's password on stdin "
                  "(or MXTRAIN_PLATFORM_PASSWORD)", file=sys.stderr)
            return 2
        idp.add_user(a.user, pw)
        plan["user_created"] = True
    dns = ["localhost"] + ([a.host] if a.host not in ("127.0.0.1", "0.0.0.0", "localhost") else [])
    cert = idp.issue_cert("dashboard", dns, ips=["127.0.0.1"])
    plan.update({"cert": cert["cert"], "ca": cert["ca"], "url": f"https://{dns[-1]}:{a.port}/"})
    print(json.dumps(plan, indent=1), flush=True)
    if a.dry_run:
        return 0
    from .mlplatform.dashboard import main as dash
    return dash(["--host", a.host, "--port", str(a.port), "--certfile", cert["cert"], "--keyfile", cert["key"],
                 "--oidc"])


def cmd_profile(a):
    from .mlplatform import profiles as pr
    if a.action == "create":
        prof = pr.create(a.name, owner=a.owner, gpu_quota=a.gpu_quota, contributors=a.contributor)
        print(json.dumps(prof, indent=1))
    elif a.action == "delete":
        pr.delete(a.name)
        print(f'profile "{a.name}" deleted')
    elif a.action == "poddefault":
        import yaml
        with open(a.file) as f:
            pd = yaml.safe_load(f)
        if pd.get("kind") == "PodDefault":    # accept the Kubernetes object form too
            spec = pd.get("spec") or {}
            pd = dict(spec, name=pd["metadata"]["name"])
        pr.set_pod_default(a.name, pd)
        print(f'poddefault "{pd.get("name")}" applied to {a.name}')
    else:
        for p in pr.list_profiles():
            spec = p.get("spec") or {}
            print(f"{p['metadata']['name']:32s} owner={(spec.get('owner') or {}).get('name')} "
                  f"quota={((spec.get('resourceQuotaSpec') or {}).get('hard') or {})} "
                  f"poddefaults={[d.get('name') for d in p.get('podDefaults') or []]}")
    return 0


def build_parser():
    p = argparse.ArgumentParser(prog="mxtrain")
    sp = p.add_subparsers(dest="cmd", required=True)
    q = sp.add_parser("install")
    q.add_argument("release")
    q.add_argument("chart")
    _add_values(q)
    q.add_argument("--wait", action="store_true", help="run in the foreground until the jobs finish")
    q.add_argument("--timeout", type=float, default=None)
    q.add_argument("--debug", action="store_true", help="print the rendered manifest (helm --debug)")
    q.add_argument("--profile", action="store_true",
                   help="torch.profiler (ROCm) trace + kernel table of a step window per rank into "
                        "$HOME/logs/<pod>/profile")
    q.add_argument("--profile-steps", default="5:8")
    q.add_argument("--debug-mode", action="store_true",
                   help="serialised kernels, synchronous HIP errors, TORCH_DISTRIBUTED_DEBUG=DETAIL, "
                        "NCCL_DEBUG=INFO, per-step inf/nan checks")
    q.set_defaults(fn=cmd_install)
    q = sp.add_parser("uninstall")
    q.add_argument("release")
    q.add_argument("-n", "--namespace", default=rel.DEFAULT_NS)
    q.set_defaults(fn=cmd_uninstall)
    q = sp.add_parser("scale", help="change the replica count of an elastic PyTorchJob")
    q.add_argument("release")
    q.add_argument("--replicas", type=int, required=True)
    q.add_argument("-n", "--namespace", default=rel.DEFAULT_NS)
    q.set_defaults(fn=cmd_scale)
    q = sp.add_parser("status")
    q.add_argument("release")
    q.add_argument("-n", "--namespace", default=rel.DEFAULT_NS)
    q.add_argument("-o", "--output", default="text")
    q.set_defaults(fn=cmd_status)
    q = sp.add_parser("list")
    q.add_argument("-n", "--namespace", default=rel.DEFAULT_NS)
    q.add_argument("-A", "--all-namespaces", action="store_true")
    q.set_defaults(fn=cmd_list)
    q = sp.add_parser("logs")
    q.add_argument("release")
    q.add_argument("--pod", default=None)
    q.add_argument("-f", "--follow", action="store_true")
    q.add_argument("-n", "--namespace", default=rel.DEFAULT_NS)
    q.set_defaults(fn=cmd_logs)
    q = sp.add_parser("template")
    q.add_argument("release")
    q.add_argument("chart")
    _add_values(q)
    q.set_defaults(fn=cmd_template)
    q = sp.add_parser("lint")
    q.add_argument("chart")
    _add_values(q)
    q.set_defaults(fn=cmd_lint)
    q = sp.add_parser("pipeline")
    q.add_argument("action", choices=["run"])
    q.add_argument("file")
    q.set_defaults(fn=cmd_pipeline)
    q = sp.add_parser("node")
    q.add_argument("action", nargs="?", default="info",
                   choices=["info", "init", "stage-data", "export", "attach-pvc"])
    q.add_argument("args", nargs="*")
    q.add_argument("-f", "--file", default=None, help="node config (infra/node.yaml) for init")
    q.add_argument("--check", action="store_true", help="run the node acceptance checks (GPUs, HBM, RCCL, PV)")
    q.add_argument("--gpus", type=int, default=None)
    q.set_defaults(fn=cmd_node)
    q = sp.add_parser("dashboard", help="central dashboard (jobs, volumes, tensorboards, HPO, pipelines)")
    q.add_argument("--host", default="127.0.0.1")
    q.add_argument("--port", type=int, default=8080)
    q.add_argument("--certfile")
    q.add_argument("--keyfile")
    q.add_argument("--htpasswd")
    q.add_argument("--oidc", action="store_true", help="bearer / session JWTs of the node identity provider")
    q.add_argument("--tls-auto", action="store_true", help="HTTPS with a certificate from the node CA")
    q.set_defaults(fn=cmd_dashboard)
    q = sp.add_parser("identity", help="identity provider users / node certificates (Dex, cert-manager roles)")
    q.add_argument("args", nargs=argparse.REMAINDER)
    q.set_defaults(fn=cmd_identity)
    q = sp.add_parser("platform", help="bring up the platform services (profile, user, certificate, dashboard)")
    q.add_argument("action", choices=["up"])
    q.add_argument("--user", default="user@example.com")
    q.add_argument("--namespace", default=rel.DEFAULT_NS)
    q.add_argument("--gpu-quota", type=int, default=None)
    q.add_argument("--host", default="127.0.0.1")
    q.add_argument("--port", type=int, default=8443)
    q.add_argument("--dry-run", action="store_true", help="set up, print the plan, do not serve")
    q.set_defaults(fn=cmd_platform)
    q = sp.add_parser("profile", help="namespaces (Kubeflow Profiles): quotas, owners, PodDefaults")
    q.add_argument("action", choices=["create", "list", "delete", "poddefault"])
    q.add_argument("name", nargs="?", default=rel.DEFAULT_NS)
    q.add_argument("--owner", default="user@example.com")
    q.add_argument("--gpu-quota", type=int, default=None)
    q.add_argument("--contributor", action="append", default=[])
    q.add_argument("-f", "--file", help="PodDefault YAML (poddefault action)")
    q.set_defaults(fn=cmd_profile)
    q = sp.add_parser("hpo")
    q.add_argument("action", choices=["run"])
    q.add_argument("file")
    q.add_argument("-n", "--namespace", default=rel.DEFAULT_NS)
    q.set_defaults(fn=cmd_hpo)
    return p


def main(argv=None):
    a = build_parser().parse_args(argv)
    sys.exit(a.fn(a))


if __name__ == "__main__":
    main()

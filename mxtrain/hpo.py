"""Hyper-parameter search over chart releases -- the single-node stand-in for Katib
(random / grid search, StdOut metrics collector, median early stopping,
trial templates that launch a PyTorchJob).

An experiment file (YAML) mirrors Katib's Experiment spec::

    name: gpt-lr
    objective: {type: minimize, objectiveMetricName: lm_loss, goal: 5.0,
                additionalMetricNames: [grad_norm]}
    algorithm: {algorithmName: random, seed: 0}            # random | grid
    parallelTrialCount: 1
    maxTrialCount: 6
    maxFailedTrialCount: 2
    earlyStopping: {algorithmName: medianstop, minTrialsRequired: 3}
    parameters:
      - {name: lr, parameterType: double, feasibleSpace: {min: "1e-5", max: "1e-3"}, scale: log}
      - {name: mbs, parameterType: categorical, feasibleSpace: {list: ["2", "4"]}}
    trialTemplate:
      chart: charts/machine-learning/training/pytorchjob-distributed
      values: [examples/.../pretrain.yaml]                   # -f files
      set: ["train.env[0].value=${trialParameters.lr}"]      # --set with substitution
      metricsCollector: {kind: StdOut, format: "(?P<name>[\\w\\s]+?):\\s*(?P<value>[-+0-9.eE]+)"}

Trials are installed as releases ``<experiment>-<n>`` and run to completion (the GPU
ledger serialises trials that would not fit); the metric is the last value the collector
finds in the trial's logs (Katib's default "latest" strategy).  Results go to
``$MXTRAIN_HOME/hpo/<name>/experiment.json`` and the best trial is printed.
"""
from __future__ import annotations

import concurrent.futures as cf
import itertools
import json
import math
import os
import random
import re
import statistics
from typing import Dict, List, Optional

import yaml

from .launch import release as rel
from .runtime.storage import mxtrain_home

DEFAULT_FORMAT = r"(?P<name>[A-Za-z_][\w \-/()]*?)\s*[:=]\s*(?P<value>[-+]?\d+\.?\d*(?:[eE][-+]?\d+)?)"


def _sample(p: dict, r: random.Random):
    fs = p.get("feasibleSpace", {})
    t = p.get("parameterType", "double")
    if t == "categorical":
        return r.choice(list(fs["list"]))
    lo, hi = float(fs["min"]), float(fs["max"])
    if p.get("scale") == "log":
        v = math.exp(r.uniform(math.log(lo), math.log(hi)))
    else:
        v = r.uniform(lo, hi)
    if t == "int":
        return str(int(round(v)))
    return f"{v:.6g}"


def _grid(p: dict) -> List[str]:
    fs = p.get("feasibleSpace", {})
    t = p.get("parameterType", "double")
    if t == "categorical":
        return [str(x) for x in fs["list"]]
    lo, hi = float(fs["min"]), float(fs["max"])
    if t == "int":
        step = int(fs.get("step", 1))
        return [str(v) for v in range(int(lo), int(hi) + 1, step)]
    step = float(fs.get("step", (hi - lo) / 4 if hi > lo else 1.0))
    out, v = [], lo
    while v <= hi + 1e-12:
        out.append(f"{v:.6g}")
        v += step
    return out


def suggestions(exp: dict):
    alg = (exp.get("algorithm") or {}).get("algorithmName", "random")
    params = exp["parameters"]
    n = int(exp.get("maxTrialCount", 10))
    if alg == "grid":
        combos = itertools.product(*[_grid(p) for p in params])
        for k, c in enumerate(combos):
            if k >= n:
                break
            yield {p["name"]: v for p, v in zip(params, c)}
    elif alg == "random":
        r = random.Random(int((exp.get("algorithm") or {}).get("seed", 0)))
        for _ in range(n):
            yield {p["name"]: _sample(p, r) for p in params}
    else:
        raise ValueError(f"algorithm {alg} not supported (random, grid)")


def _subst(s: str, params: Dict[str, str]) -> str:
    return re.sub(r"\$\{trialParameters\.([A-Za-z0-9_]+)\}", lambda m: params[m.group(1)], s)


def collect(text: str, names: List[str], fmt: Optional[str] = None) -> Dict[str, float]:
    rx = re.compile(fmt or DEFAULT_FORMAT)
    want = {n.lower().replace(" ", "_"): n for n in names}
    out: Dict[str, float] = {}
    for line in text.splitlines():
        for m in rx.finditer(line):
            key = m.group("name").strip().lower().replace(" ", "_")
            # "step 10 loss: 4.5" reports metric "loss"; "lm loss: ..." reports "lm_loss"
            hit = key if key in want else next((w for w in want if key.endswith("_" + w)), None)
            if hit is not None:
                try:
                    out[want[hit]] = float(m.group("value"))
                except ValueError:
                    pass
    return out


def run_experiment(exp: dict, namespace: str = rel.DEFAULT_NS, log=print) -> dict:
    name = exp["name"]
    obj = exp["objective"]
    metric = obj["objectiveMetricName"]
    names = [metric] + list(obj.get("additionalMetricNames") or [])
    minimize = obj.get("type", "minimize") == "minimize"
    goal = obj.get("goal")
    tmpl = exp["trialTemplate"]
    fmt = (tmpl.get("metricsCollector") or {}).get("format")
    es = exp.get("earlyStopping") or {}
    out_dir = os.path.join(mxtrain_home(), "hpo", name)
    os.makedirs(out_dir, exist_ok=True)
    trials: List[dict] = []
    failed = 0

    def one(k: int, params: Dict[str, str]) -> dict:
        rname = f"{name}-{k}"
        sets = [_subst(s, params) for s in tmpl.get("set", [])]
        st = rel.install(tmpl["chart"], rname, namespace, list(tmpl.get("values", [])), sets, wait=True,
                         timeout=tmpl.get("timeout"))
        text = rel.logs(rname, namespace)
        m = collect(text, names, fmt)
        rec = {"trial": rname, "parameters": params, "phase": st["phase"], "metrics": m}
        rel.uninstall(rname, namespace, keep_history=True)
        return rec

    par = max(1, int(exp.get("parallelTrialCount", 1)))
    sug = list(suggestions(exp))
    with cf.ThreadPoolExecutor(max_workers=par) as ex:
        futs = {}
        k = 0
        while k < len(sug) or futs:
            while k < len(sug) and len(futs) < par:
                futs[ex.submit(one, k, sug[k])] = k
                k += 1
            done, _ = cf.wait(list(futs), return_when=cf.FIRST_COMPLETED)
            for f in done:
                futs.pop(f)
                rec = f.result()
                v = rec["metrics"].get(metric)
                if rec["phase"] != "Succeeded" or v is None:
                    rec["status"] = "Failed"
                    failed += 1
                else:
                    rec["status"] = "Succeeded"
                    # median stopping: a finished trial worse than the median of the completed
                    # ones is marked EarlyStopped (it does not become the best)
                    done_vals = [t["metrics"][metric] for t in trials if t.get("status") == "Succeeded"]
                    if es.get("algorithmName") == "medianstop" and len(done_vals) >= int(es.get("minTrialsRequired", 3)):
                        med = statistics.median(done_vals)
                        if (v > med) if minimize else (v < med):
                            rec["status"] = "EarlyStopped"
                trials.append(rec)
                log(f"[hpo] {rec['trial']} {rec['parameters']} -> {rec['status']} {rec['metrics']}")
                if failed > int(exp.get("maxFailedTrialCount", len(sug))):
                    k = len(sug)
                if goal is not None and v is not None and ((v <= goal) if minimize else (v >= goal)):
                    k = len(sug)     # goal reached: stop scheduling new trials
    good = [t for t in trials if t.get("status") == "Succeeded"]
    best = (min if minimize else max)(good, key=lambda t: t["metrics"][metric]) if good else None
    res = {"name": name, "objective": obj, "trials": trials, "best": best,
           "condition": "Succeeded" if best else "Failed"}
    with open(os.path.join(out_dir, "experiment.json"), "w") as f:
        json.dump(res, f, indent=1)
    return res


def load_experiment(path: str) -> dict:
    with open(path) as f:
        return yaml.safe_load(f)

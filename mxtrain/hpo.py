"""Hyper-parameter and architecture search over chart releases -- the single-node
stand-in for Katib.  Suggestion algorithms: random, grid, sobol, tpe,
multivariate-tpe, bayesianoptimization, cmaes, hyperband, pbt, enas, darts
(mxtrain/katib/suggest.py; reference charts/ml-platform/kubeflow-katib/templates/
config_maps.yaml:26-64).  Metrics collectors: StdOut, File (TEXT/JSON), TensorFlowEvent
(mxtrain/katib/collectors.py; config_maps.yaml:9-25).  Early stopping: medianstop.

An experiment file (YAML) mirrors Katib's Experiment spec::

    name: gpt-lr
    objective: {type: minimize, objectiveMetricName: lm_loss, goal: 5.0,
                additionalMetricNames: [grad_norm],
                metricStrategies: [{name: lm_loss, value: latest}]}   # default: min/max
    algorithm: {algorithmName: tpe, algorithmSettings: [{name: random_state, value: "1"}]}
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
    metricsCollectorSpec:                                    # default StdOut
      collector: {kind: File}
      source: {fileSystemPath: {path: /efs/hpo/${trialName}/metrics.jsonl, format: JSON}}

``${trialParameters.<name>}`` and ``${trialName}`` are substituted into the template's
``set`` values and the collector path.  Trials are installed as releases ``<name>-<n>``
and run to completion (the GPU ledger serialises trials that would not fit).  Adaptive
algorithms see every finished trial before their next suggestion; rung/generation based
ones (hyperband, cmaes, pbt) wait for the running trials when they need their results.
Results go to ``$MXTRAIN_HOME/hpo/<name>/experiment.json``.
"""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import re
import statistics
from typing import Dict, List, Optional

import yaml

from .katib import collectors as kc
from .katib.suggest import WAIT, make_suggester
from .launch import release as rel
from .runtime.storage import mxtrain_home

DEFAULT_FORMAT = kc.DEFAULT_FORMAT


def suggestions(exp: dict):
    """All suggestions of a non-adaptive algorithm (random / grid / sobol)."""
    s = make_suggester(exp)
    while True:
        p = s.ask([])
        if p is None or p is WAIT:
            return
        yield p


def _subst(s: str, params: Dict[str, str], trial: str = "") -> str:
    s = re.sub(r"\$\{trialParameters\.([A-Za-z0-9_\-]+)\}", lambda m: str(params[m.group(1)]), s)
    return s.replace("${trialName}", trial).replace("${trialSpec.Name}", trial)


def collect(text: str, names: List[str], fmt: Optional[str] = None) -> Dict[str, float]:
    """StdOut collector with the ``latest`` strategy (kept for callers of the old API)."""
    return {k: v[-1] for k, v in kc.parse_text(text, names, fmt).items()}


def _collector_spec(exp: dict) -> dict:
    mc = exp.get("metricsCollectorSpec")
    if mc:
        return mc
    old = (exp.get("trialTemplate") or {}).get("metricsCollector") or {}
    return {"collector": {"kind": old.get("kind", "StdOut")}, "format": old.get("format"),
            "source": old.get("source")}


def run_experiment(exp: dict, namespace: str = rel.DEFAULT_NS, log=print) -> dict:
    name = exp["name"]
    obj = exp["objective"]
    metric = obj["objectiveMetricName"]
    names = [metric] + list(obj.get("additionalMetricNames") or [])
    strat = kc.strategies(obj)
    minimize = obj.get("type", "minimize") == "minimize"
    goal = obj.get("goal")
    tmpl = exp["trialTemplate"]
    mc = _collector_spec(exp)
    es = exp.get("earlyStopping") or {}
    out_dir = os.path.join(mxtrain_home(), "hpo", name)
    os.makedirs(out_dir, exist_ok=True)
    sug = make_suggester(exp, root=out_dir)
    trials: List[dict] = []
    history: List[dict] = []
    failed = 0
    max_failed = int(exp.get("maxFailedTrialCount", 10 ** 9))

    def one(k: int, params: Dict[str, str]) -> dict:
        rname = f"{name}-{k}"
        sets = [_subst(s, params, rname) for s in tmpl.get("set", [])]
        st = rel.install(tmpl["chart"], rname, namespace, list(tmpl.get("values", [])), sets, wait=True,
                         timeout=tmpl.get("timeout"))
        text = rel.logs(rname, namespace)
        obs = kc.collect(mc, names, text, lambda s: _subst(s, params, rname))
        rec = {"trial": rname, "parameters": params, "phase": st["phase"], "metrics": kc.reduce(obs, strat),
               "observations": {k2: len(v) for k2, v in obs.items()}}
        rel.uninstall(rname, namespace, keep_history=True)
        return rec

    par = max(1, int(exp.get("parallelTrialCount", 1)))
    stop = False
    k = 0
    with cf.ThreadPoolExecutor(max_workers=par) as ex:
        futs = {}
        while True:
            while not stop and len(futs) < par:
                p = sug.ask(history)
                if p is None:
                    stop = True
                    break
                if p is WAIT:
                    break
                futs[ex.submit(one, k, p)] = k
                k += 1
            if not futs:
                break
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
                history.append({"name": rec["trial"], "parameters": rec["parameters"], "value": v,
                                "status": rec["status"]})
                log(f"[hpo] {rec['trial']} {rec['parameters']} -> {rec['status']} {rec['metrics']}")
                if failed > max_failed:
                    stop = True
                if goal is not None and v is not None and ((v <= goal) if minimize else (v >= goal)):
                    stop = True      # goal reached: stop scheduling new trials
    good = [t for t in trials if t.get("status") == "Succeeded"]
    best = (min if minimize else max)(good, key=lambda t: t["metrics"][metric]) if good else None
    res = {"name": name, "objective": obj, "algorithm": (exp.get("algorithm") or {}).get("algorithmName", "random"),
           "trials": trials, "best": best, "condition": "Succeeded" if best else "Failed"}
    with open(os.path.join(out_dir, "experiment.json"), "w") as f:
        json.dump(res, f, indent=1)
    return res


def load_experiment(path: str) -> dict:
    with open(path) as f:
        return yaml.safe_load(f)

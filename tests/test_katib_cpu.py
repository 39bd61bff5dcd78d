"""Katib-equivalent search: every suggestion algorithm the reference's katib-config lists
(charts/ml-platform/kubeflow-katib/templates/config_maps.yaml:26-64) driven on a
synthetic objective, the three metrics collectors (:9-25) and metric strategies, plus an
end-to-end experiment through a chart with a File collector."""
import json
import os
import re

import numpy as np
import pytest

from mxtrain.katib import WAIT, make_suggester
from mxtrain.katib import collectors as kc

XY = [{"name": "x", "parameterType": "double", "feasibleSpace": {"min": "-1", "max": "1"}},
      {"name": "y", "parameterType": "double", "feasibleSpace": {"min": "-1", "max": "1"}}]


def bowl(p):
    return (float(p["x"]) - 0.3) ** 2 + (float(p["y"]) + 0.2) ** 2


def drive(exp, f, par=1, root="."):
    """Katib controller loop in miniature: keep `par` trials running, finish the oldest."""
    s = make_suggester(exp, root=root)
    hist, running = [], []
    for _ in range(10000):
        while len(running) < par:
            p = s.ask(hist)
            if p is None or p is WAIT:
                break
            running.append(p)
        if not running:
            return hist
        p = running.pop(0)
        hist.append({"name": f"t{len(hist)}", "parameters": p, "value": f(p), "status": "Succeeded"})
    raise AssertionError("suggester did not terminate")


def exp_of(alg, n, params=XY, settings=(), **kw):
    e = {"name": alg, "objective": {"type": "minimize", "objectiveMetricName": "loss"},
         "algorithm": {"algorithmName": alg,
                       "algorithmSettings": [{"name": k, "value": str(v)} for k, v in settings]},
         "maxTrialCount": n, "parameters": params}
    e.update(kw)
    return e


@pytest.mark.parametrize("alg", ["tpe", "multivariate-tpe", "bayesianoptimization", "cmaes"])
def test_model_based_algorithms_improve(alg):
    hist = drive(exp_of(alg, 48, settings=[("random_state", 3)]), bowl, par=2)
    vals = [h["value"] for h in hist]
    assert len(vals) == 48
    assert min(vals[:32]) < 0.03, (alg, vals)       # random search's best of 48 is ~0.035 here
    if alg != "bayesianoptimization":               # EI explores once the optimum is pinned
        assert np.mean(vals[-12:]) < 0.5 * np.mean(vals[:12]), (alg, vals)


def test_random_grid_sobol():
    r = drive(exp_of("random", 10, settings=[("random_state", 1)]), bowl)
    assert len(r) == 10 and all(-1 <= float(h["parameters"]["x"]) <= 1 for h in r)
    g = drive(exp_of("grid", 100, params=[{"name": "x", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "3"}},
                                          {"name": "c", "parameterType": "categorical",
                                           "feasibleSpace": {"list": ["a", "b"]}}]), lambda p: 0.0)
    assert [(h["parameters"]["x"], h["parameters"]["c"]) for h in g] == \
        [("1", "a"), ("1", "b"), ("2", "a"), ("2", "b"), ("3", "a"), ("3", "b")]
    s = drive(exp_of("sobol", 16, settings=[("random_state", 0)]), bowl)
    quad = [(float(h["parameters"]["x"]) > 0, float(h["parameters"]["y"]) > 0) for h in s]
    assert all(quad.count(q) == 4 for q in set(quad)) and len(set(quad)) == 4   # balanced (0,m,2)-net


def test_hyperband_brackets_and_promotion():
    params = XY[:1] + [{"name": "epochs", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "9"}}]
    e = exp_of("hyperband", 1000, params=params, settings=[("resource_name", "epochs"), ("eta", 3), ("r_l", 9)])
    hist = drive(e, lambda p: abs(float(p["x"]) - 0.3) / float(p["epochs"]), par=3)
    res = [int(h["parameters"]["epochs"]) for h in hist]
    # R=9, eta=3: brackets s=2 (9@1, 3@3, 1@9), s=1 (5@3, 1@9), s=0 (3@9)
    assert res == [1] * 9 + [3] * 3 + [9] + [3] * 5 + [9] + [9] * 3
    rung0 = hist[:9]
    best3 = sorted(rung0, key=lambda h: h["value"])[:3]
    assert {h["parameters"]["x"] for h in hist[9:12]} == {h["parameters"]["x"] for h in best3}


def test_pbt_exploit_explore(tmp_path):
    e = exp_of("pbt", 12, params=[XY[0], {"name": "bs", "parameterType": "categorical",
                                           "feasibleSpace": {"list": ["8", "16"]}}],
               settings=[("n_population", 4), ("truncation_threshold", 0.25), ("random_state", 2)])
    hist = drive(e, lambda p: abs(float(p["x"]) - 0.3), par=4, root=str(tmp_path))
    assert len(hist) == 12
    g0, g1 = hist[:4], hist[4:8]
    assert all(h["parameters"]["parent_checkpoint_dir"] == "" for h in g0)
    ck0 = {h["parameters"]["checkpoint_dir"] for h in g0}
    assert all(h["parameters"]["parent_checkpoint_dir"] in ck0 for h in g1)
    best0 = min(g0, key=lambda h: h["value"])["parameters"]["checkpoint_dir"]
    worst0 = max(g0, key=lambda h: h["value"])["parameters"]["checkpoint_dir"]
    parents = [h["parameters"]["parent_checkpoint_dir"] for h in g1]
    assert parents.count(best0) == 2 and worst0 not in parents     # the worst exploits the best
    assert len({h["parameters"]["checkpoint_dir"] for h in hist}) == 12


def _op(t, sizes=None):
    if sizes is None:
        return {"operationType": t}
    return {"operationType": t, "parameters": [{"name": "filter_size", "parameterType": "categorical",
                                                 "feasibleSpace": {"list": sizes}}]}


NAS = {"graphConfig": {"numLayers": 4, "inputSizes": [32, 32, 3], "outputSizes": [10]},
       "operations": [_op("separable_convolution", ["3", "5"]), _op("max_pooling", ["3"])]}


def test_enas_controller_learns():
    e = {"name": "enas", "objective": {"type": "maximize", "objectiveMetricName": "acc"},
         "algorithm": {"algorithmName": "enas", "algorithmSettings": [{"name": "controller_learning_rate",
                                                                        "value": "0.5"}]},
         "maxTrialCount": 80, "nasConfig": NAS}

    def reward(p):   # best architecture: op 0 (conv 3x3) everywhere, no skips
        arch = json.loads(p["architecture"])
        return sum(l[0] == 0 for l in arch) - 0.5 * sum(sum(l[1:]) for l in arch)
    hist = drive(e, reward)
    cfg = json.loads(hist[0]["parameters"]["nn_config"])
    assert cfg["num_layers"] == 4 and len(cfg["embedding"]) == 3
    arch = json.loads(hist[0]["parameters"]["architecture"])
    assert [len(l) for l in arch] == [1, 2, 3, 4]
    vals = [h["value"] for h in hist]
    assert np.mean(vals[-20:]) > np.mean(vals[:20]) + 0.5


def test_darts_single_trial():
    e = {"name": "darts", "objective": {"type": "maximize", "objectiveMetricName": "Best-Genotype"},
         "algorithm": {"algorithmName": "darts", "algorithmSettings": [{"name": "num_epochs", "value": "2"}]},
         "maxTrialCount": 5, "nasConfig": NAS}
    hist = drive(e, lambda p: 0.0)
    assert len(hist) == 1
    p = hist[0]["parameters"]
    assert json.loads(p["algorithm-settings"]) == {"num_epochs": "2"} and p["num-layers"] == "4"
    assert json.loads(p["search-space"]) == ["max_pooling_3x3", "separable_convolution_3x3",
                                             "separable_convolution_5x5"]


def test_collectors_and_strategies(tmp_path):
    names = ["loss", "acc"]
    text = "epoch 1 loss=0.9 acc=0.5\nepoch 2 loss: 0.4 acc: 0.7\nepoch 3 loss=0.6 acc=0.65\n"
    obs = kc.parse_text(text, names)
    assert obs == {"loss": [0.9, 0.4, 0.6], "acc": [0.5, 0.7, 0.65]}
    st = kc.strategies({"type": "minimize", "objectiveMetricName": "loss", "additionalMetricNames": ["acc"]})
    assert kc.reduce(obs, st) == {"loss": 0.4, "acc": 0.65}
    st2 = kc.strategies({"type": "minimize", "objectiveMetricName": "loss",
                         "metricStrategies": [{"name": "loss", "value": "latest"}]})
    assert kc.reduce(obs, st2)["loss"] == 0.6
    # Katib-style positional-group regex
    assert kc.parse_text("loss=1.5", ["loss"], r"([\w|-]+)\s*=\s*([+-]?\d*(\.\d+)?([Ee][+-]?\d+)?)") == {"loss": [1.5]}
    # File / JSON
    f = tmp_path / "m.jsonl"
    f.write_text('{"loss": 2.0, "step": 1}\nnot json\n{"loss": 1.0, "acc": 0.9}\n')
    mc = {"collector": {"kind": "File"}, "source": {"fileSystemPath": {"path": str(f), "format": "JSON"}}}
    assert kc.collect(mc, names, "") == {"loss": [2.0, 1.0], "acc": [0.9]}
    # TensorFlowEvent
    from mxtrain.obs.tensorboard import SummaryWriter
    d = tmp_path / "tb"
    with SummaryWriter(str(d)) as w:
        for step, v in ((2, 0.3), (1, 0.8), (3, 0.5)):
            w.add_scalar("train/loss", v, step)
    mc = {"collector": {"kind": "TensorFlowEvent"}, "source": {"fileSystemPath": {"path": str(d), "kind": "Directory"}}}
    got = kc.collect(mc, ["loss"], "")
    assert got["loss"] == pytest.approx([0.8, 0.3, 0.5])


@pytest.fixture
def home(tmp_path, monkeypatch):
    monkeypatch.setenv("MXTRAIN_HOME", str(tmp_path / "home"))
    monkeypatch.setenv("MXTRAIN_FAKE_GPUS", "8")
    return tmp_path


def test_experiment_file_collector_tpe(home, tmp_path):
    """TPE experiment over the data-process chart; each trial writes JSON metric lines to a
    per-trial file (${trialName} in the path) that the File collector reads."""
    from mxtrain.hpo import run_experiment
    charts = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "charts",
                          "machine-learning", "data-prep", "data-process")
    mdir = tmp_path / "metrics"
    mdir.mkdir()
    # (no commas: --set splits on them)
    prog = ("import json;import pathlib;x=${trialParameters.x};pathlib.Path('%s/${trialName}.jsonl').write_text("
            "chr(10).join(json.dumps({'loss': (x-3)**2+0.5+1.0/(s+1)}) for s in range(3)))" % mdir)
    exp = {"name": "tpe-file", "objective": {"type": "minimize", "objectiveMetricName": "loss"},
           "algorithm": {"algorithmName": "tpe", "algorithmSettings": [{"name": "n_startup_trials", "value": "3"}]},
           "parallelTrialCount": 2, "maxTrialCount": 6,
           "parameters": [{"name": "x", "parameterType": "int", "feasibleSpace": {"min": "1", "max": "5"}}],
           "metricsCollectorSpec": {"collector": {"kind": "File"},
                                    "source": {"fileSystemPath": {"path": str(mdir / "${trialName}.jsonl"),
                                                                  "format": "JSON"}}},
           "trialTemplate": {"chart": charts,
                             "set": ["process.command[0]=python3", "process.args[0]=-c",
                                     f"process.args[1]=\"{prog}\""]}}
    res = run_experiment(exp, log=lambda *a: None)
    assert res["condition"] == "Succeeded" and len(res["trials"]) == 6
    for t in res["trials"]:
        x = int(t["parameters"]["x"])
        assert t["metrics"]["loss"] == pytest.approx((x - 3) ** 2 + 0.5 + 1.0 / 3)   # min over the 3 lines
        assert t["observations"]["loss"] == 3


def test_darts_trial_runs(capsys):
    """The trial side of DARTS: a first-order search over the suggested primitives prints the
    genotype and validation accuracy for the StdOut collector."""
    from mxtrain.workloads.nas.darts import main
    prims = ["separable_convolution_3x3", "max_pooling_3x3", "skip_connection"]
    assert main(["--num-layers", "2", "--samples", "64", "--search-space", json.dumps(prims),
                 "--algorithm-settings", json.dumps({"num_epochs": "1", "batch_size": "32"})]) == 0
    out = capsys.readouterr().out
    geno = json.loads(re.search(r"Best-Genotype=(.*)", out).group(1))
    assert len(geno) == 2 and all(len(c) == 3 and set(c) <= set(prims) for c in geno)
    assert kc.parse_text(out, ["Validation-accuracy"])["Validation-accuracy"]

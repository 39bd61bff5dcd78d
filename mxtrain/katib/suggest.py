"""Katib suggestion algorithms, in-process.

The reference deploys one suggestion service per algorithm
(charts/ml-platform/kubeflow-katib/templates/config_maps.yaml:26-64: random, tpe, grid,
hyperband, bayesianoptimization, cmaes, sobol, multivariate-tpe, enas, darts, pbt).  Here
each is a class with Katib's ask/tell contract collapsed into one call:

    s = make_suggester(exp)              # exp = Experiment spec (dict)
    s.ask(history) -> dict | WAIT | None # next trial's assignments; WAIT = needs results
                                         # of running trials first; None = search done

``history`` is the list of finished trials, each ``{"name", "parameters", "value",
"status"}`` (value = the objective metric, None when the trial failed).  Every
algorithm optimises ``loss = value`` (minimize) or ``-value`` (maximize); settings come
from ``algorithm.algorithmSettings`` (Katib's name/value list) with Katib's names.

Algorithms are implemented from their published descriptions with numpy / scipy only
(hyperopt, optuna, skopt, goptuna are not installed): TPE (Bergstra et al. 2011),
multivariate TPE (Falkner et al. 2018 product kernel), GP-EI Bayesian optimisation,
CMA-ES (Hansen 2016 tutorial), scrambled Sobol (scipy.stats.qmc), Hyperband
(Li et al. 2018), PBT (Jaderberg et al. 2017), ENAS-style REINFORCE controller
(Pham et al. 2018, per-decision softmax policy), DARTS (the search runs inside one trial,
mxtrain.workloads.nas.darts).
"""
from __future__ import annotations

import itertools
import json
import math
import random
from typing import Dict, List, Optional

import numpy as np

from .space import Space

WAIT = "wait"


def settings_of(exp: dict) -> Dict[str, str]:
    alg = exp.get("algorithm") or {}
    out = {s["name"]: s.get("value") for s in alg.get("algorithmSettings") or []}
    if "seed" in alg and "random_state" not in out:
        out["random_state"] = alg["seed"]
    return out


class Suggester:
    name = "base"

    def __init__(self, exp: dict):
        self.exp = exp
        self.space = Space(exp["parameters"]) if exp.get("parameters") else None
        self.settings = settings_of(exp)
        obj = exp.get("objective") or {}
        self.minimize = obj.get("type", "minimize") == "minimize"
        self.max_trials = int(exp.get("maxTrialCount", 10))
        seed = self.settings.get("random_state", self.settings.get("seed", 0))
        self.rng = random.Random(int(seed or 0))
        self.nrng = np.random.default_rng(int(seed or 0))
        self.issued = 0

    def setting(self, name, default, cast=float):
        v = self.settings.get(name)
        return default if v in (None, "") else cast(v)

    def loss(self, t: dict) -> Optional[float]:
        v = t.get("value")
        if v is None or t.get("status") not in ("Succeeded", "EarlyStopped"):
            return None
        return float(v) if self.minimize else -float(v)

    def ask(self, history: List[dict]):
        if self.issued >= self.max_trials:
            return None
        s = self._ask(history)
        if s is not None and s is not WAIT:
            self.issued += 1
        return s

    def _ask(self, history):
        raise NotImplementedError


class RandomSearch(Suggester):
    name = "random"

    def _ask(self, history):
        return self.space.sample(self.rng)


class GridSearch(Suggester):
    name = "grid"

    def __init__(self, exp):
        super().__init__(exp)
        self.it = itertools.product(*[d.grid() for d in self.space.dims])

    def _ask(self, history):
        c = next(self.it, None)
        return None if c is None else dict(zip(self.space.names, c))


class SobolSearch(Suggester):
    name = "sobol"

    def __init__(self, exp):
        super().__init__(exp)
        from scipy.stats import qmc
        self.q = qmc.Sobol(len(self.space), scramble=True, seed=int(self.settings.get("random_state") or 0))

    def _ask(self, history):
        return self.space.from_unit(self.q.random(1)[0])


# ------------------------------------------------------------------------------ TPE
class TPE(Suggester):
    """Tree-structured Parzen estimator.  Finished trials are split at the ``gamma``
    quantile of the loss into good (l) and bad (g) sets; each set becomes an adaptive
    Parzen mixture (hyperopt's estimator: one Gaussian per observation with a bandwidth
    from its neighbour gaps, plus a wide prior component), candidates are drawn from l
    and the one maximising l(x)/g(x) is suggested.  ``multivariate`` (optuna's
    multivariate TPE) uses each observation as one joint component across parameters
    instead of independent per-parameter mixtures."""
    name = "tpe"

    def __init__(self, exp, multivariate: bool = False):
        super().__init__(exp)
        self.multivariate = multivariate
        self.n_startup = int(self.setting("n_startup_trials", 10))
        self.n_cand = int(self.setting("n_ei_candidates", 24))
        self.gamma = self.setting("gamma", 0.25)
        self.prior_weight = self.setting("prior_weight", 1.0)

    def _obs(self, history):
        xs, ys = [], []
        for t in history:
            y = self.loss(t)
            if y is not None:
                xs.append(self.space.to_unit(t["parameters"]))
                ys.append(y)
        return np.asarray(xs, dtype=np.float64).reshape(len(xs), len(self.space)), np.asarray(ys)

    def _parzen(self, pts: np.ndarray):
        """-> (mus, sigmas, weights); the last component is the prior N(0.5, 1)."""
        n = len(pts)
        if n == 0:
            return np.array([0.5]), np.array([1.0]), np.array([1.0])
        order = np.argsort(pts, kind="mergesort")
        srt = pts[order]
        left = np.diff(np.concatenate([[0.0], srt]))
        right = np.diff(np.concatenate([srt, [1.0]]))
        sig_s = np.maximum(left, right)
        sig = np.empty(n)
        sig[order] = sig_s
        sig = np.clip(sig, 1.0 / min(100.0, n + 1.0), 1.0)
        mus = np.concatenate([pts, [0.5]])
        sigmas = np.concatenate([sig, [1.0]])
        w = np.concatenate([np.ones(n), [self.prior_weight]])
        return mus, sigmas, w / w.sum()

    @staticmethod
    def _mix_logpdf(x: np.ndarray, mus, sigmas, w) -> np.ndarray:
        z = (x[:, None] - mus[None, :]) / sigmas[None, :]
        lp = -0.5 * z * z - np.log(sigmas[None, :] * math.sqrt(2 * math.pi)) + np.log(w[None, :])
        m = lp.max(1, keepdims=True)
        return m[:, 0] + np.log(np.exp(lp - m).sum(1))

    def _cat_probs(self, pts: np.ndarray, k: int) -> np.ndarray:
        pi = np.minimum((pts * k).astype(int), k - 1)
        cnt = np.bincount(pi, minlength=k).astype(np.float64) + self.prior_weight
        return cnt / cnt.sum()

    def _ask(self, history):
        X, y = self._obs(history)
        if len(y) < self.n_startup:
            return self.space.sample(self.rng)
        n_good = max(1, int(math.ceil(self.gamma * len(y))))
        order = np.argsort(y, kind="mergesort")
        good, bad = X[order[:n_good]], X[order[n_good:]]
        if len(bad) == 0:
            bad = X
        D = len(self.space)
        if not self.multivariate:
            u = np.empty(D)
            for j, d in enumerate(self.space.dims):
                if d.choices is not None:
                    k = d.n_choices
                    pl, pg = self._cat_probs(good[:, j], k), self._cat_probs(bad[:, j], k)
                    idx = self.nrng.choice(k, size=self.n_cand, p=pl)
                    best = idx[int(np.argmax(np.log(pl[idx]) - np.log(pg[idx])))]
                    u[j] = (best + 0.5) / k
                    continue
                ml, sl, wl = self._parzen(good[:, j])
                comp = self.nrng.choice(len(wl), size=self.n_cand, p=wl)
                c = np.clip(ml[comp] + sl[comp] * self.nrng.standard_normal(self.n_cand), 0.0, 1.0)
                score = self._mix_logpdf(c, ml, sl, wl) - self._mix_logpdf(c, *self._parzen(bad[:, j]))
                u[j] = c[int(np.argmax(score))]
            return self.space.from_unit(u)
        # multivariate: component i = observation i in every dimension (last = prior)
        comps_l = [self._parzen(good[:, j]) for j in range(D)]
        comps_g = [self._parzen(bad[:, j]) for j in range(D)]
        wl = comps_l[0][2]
        pick = self.nrng.choice(len(wl), size=self.n_cand, p=wl)
        cand = np.empty((self.n_cand, D))
        for j, d in enumerate(self.space.dims):
            mus, sig, _ = comps_l[j]
            if d.choices is not None:
                k = d.n_choices
                own = np.minimum((mus[pick] * k).astype(int), k - 1)
                rnd = self.nrng.integers(0, k, size=self.n_cand)
                keep = (self.nrng.random(self.n_cand) < 0.75) & (pick < len(mus) - 1)
                cand[:, j] = (np.where(keep, own, rnd) + 0.5) / k
            else:
                cand[:, j] = np.clip(mus[pick] + sig[pick] * self.nrng.standard_normal(self.n_cand), 0, 1)

        def joint(c, comps):
            w = comps[0][2]
            lp = np.log(w)[None, :].repeat(len(c), 0)
            for j, d in enumerate(self.space.dims):
                mus, sig, _ = comps[j]
                if d.choices is not None:
                    k = d.n_choices
                    same = (np.minimum((c[:, j] * k).astype(int), k - 1)[:, None]
                            == np.minimum((mus * k).astype(int), k - 1)[None, :])
                    p_same = np.where(np.arange(len(mus)) < len(mus) - 1, 0.75 + 0.25 / k, 1.0 / k)
                    p_diff = np.where(np.arange(len(mus)) < len(mus) - 1, 0.25 / k, 1.0 / k)
                    lp += np.log(np.where(same, p_same[None, :], p_diff[None, :]))
                else:
                    z = (c[:, j][:, None] - mus[None, :]) / sig[None, :]
                    lp += -0.5 * z * z - np.log(sig[None, :] * math.sqrt(2 * math.pi))
            m = lp.max(1, keepdims=True)
            return m[:, 0] + np.log(np.exp(lp - m).sum(1))

        score = joint(cand, comps_l) - joint(cand, comps_g)
        return self.space.from_unit(cand[int(np.argmax(score))])


# ------------------------------------------------------------------------------ GP-EI
class BayesOpt(Suggester):
    """Gaussian-process Bayesian optimisation (skopt's default family): Matern-5/2 GP on
    the unit cube (categoricals one-hot), hyper-parameters by a small marginal-likelihood
    grid, expected-improvement acquisition maximised over random + local candidates."""
    name = "bayesianoptimization"

    def __init__(self, exp):
        super().__init__(exp)
        self.n_init = int(self.setting("n_initial_points", 10))
        self.n_cand = int(self.setting("n_candidates", 2000))
        self.xi = self.setting("xi", 0.01)

    def _enc(self, U: np.ndarray) -> np.ndarray:
        cols = []
        for j, d in enumerate(self.space.dims):
            if d.categorical:
                k = d.n_choices
                idx = np.minimum((U[:, j] * k).astype(int), k - 1)
                cols.append(np.eye(k)[idx] / math.sqrt(2))
            else:
                cols.append(U[:, j:j + 1])
        return np.concatenate(cols, axis=1)

    @staticmethod
    def _matern(A, B, ls):
        d = np.sqrt(np.maximum(((A[:, None, :] - B[None, :, :]) ** 2).sum(-1), 0)) / ls
        return (1 + math.sqrt(5) * d + 5.0 / 3.0 * d * d) * np.exp(-math.sqrt(5) * d)

    def _ask(self, history):
        xs, ys = [], []
        for t in history:
            y = self.loss(t)
            if y is not None:
                xs.append(self.space.to_unit(t["parameters"]))
                ys.append(y)
        if len(ys) < self.n_init:
            return self.space.sample(self.rng)
        X = self._enc(np.asarray(xs))
        y = np.asarray(ys, dtype=np.float64)
        mu_y, sd_y = y.mean(), y.std() or 1.0
        yn = (y - mu_y) / sd_y
        best = None
        for ls in (0.1, 0.2, 0.4, 0.8, 1.6, 3.2):
            for noise in (1e-6, 1e-3, 1e-1):
                K = self._matern(X, X, ls) + noise * np.eye(len(X))
                try:
                    L = np.linalg.cholesky(K)
                except np.linalg.LinAlgError:
                    continue
                a = np.linalg.solve(L.T, np.linalg.solve(L, yn))
                nll = 0.5 * yn @ a + np.log(np.diag(L)).sum()
                if best is None or nll < best[0]:
                    best = (nll, ls, L, a)
        if best is None:
            return self.space.sample(self.rng)
        _, ls, L, a = best
        U = np.asarray(xs)
        inc = U[int(np.argmin(y))]
        cand = np.concatenate([self.nrng.random((self.n_cand, len(self.space))),
                               np.clip(inc + 0.05 * self.nrng.standard_normal((self.n_cand // 4, len(self.space))),
                                       0, 1)])
        C = self._enc(cand)
        Ks = self._matern(C, X, ls)
        mu = Ks @ a
        v = np.linalg.solve(L, Ks.T)
        var = np.maximum(1.0 - (v * v).sum(0), 1e-12)
        sd = np.sqrt(var)
        from scipy.stats import norm
        imp = yn.min() - mu - self.xi
        z = imp / sd
        ei = imp * norm.cdf(z) + sd * norm.pdf(z)
        return self.space.from_unit(cand[int(np.argmax(ei))])


# ------------------------------------------------------------------------------ CMA-ES
class CMAES(Suggester):
    """(mu/mu_w, lambda)-CMA-ES on the unit cube; one generation of ``lambda`` trials is
    handed out, then the suggester WAITs for all of them before updating the mean, step
    size and covariance."""
    name = "cmaes"

    def __init__(self, exp):
        super().__init__(exp)
        n = len(self.space)
        self.n = n
        self.lam = int(self.setting("population_size", 4 + int(3 * math.log(max(n, 1)))))
        self.mu = self.lam // 2
        w = np.log(self.mu + 0.5) - np.log(np.arange(1, self.mu + 1))
        self.w = w / w.sum()
        self.mueff = 1.0 / (self.w ** 2).sum()
        self.cc = (4 + self.mueff / n) / (n + 4 + 2 * self.mueff / n)
        self.cs = (self.mueff + 2) / (n + self.mueff + 5)
        self.c1 = 2 / ((n + 1.3) ** 2 + self.mueff)
        self.cmu = min(1 - self.c1, 2 * (self.mueff - 2 + 1 / self.mueff) / ((n + 2) ** 2 + self.mueff))
        self.damps = 1 + 2 * max(0, math.sqrt((self.mueff - 1) / (n + 1)) - 1) + self.cs
        self.chin = math.sqrt(n) * (1 - 1 / (4 * n) + 1 / (21 * n * n))
        self.mean = np.full(n, 0.5)
        self.sigma = self.setting("sigma", 0.3)
        self.C = np.eye(n)
        self.pc = np.zeros(n)
        self.ps = np.zeros(n)
        self.gen: List[tuple] = []      # (params, z-vector y) of the current generation
        self.handed = 0
        self.generation = 0

    def _new_generation(self):
        D, B = np.linalg.eigh(self.C)
        D = np.sqrt(np.maximum(D, 1e-20))
        self.gen = []
        for _ in range(self.lam):
            z = self.nrng.standard_normal(self.n)
            yv = B @ (D * z)
            x = np.clip(self.mean + self.sigma * yv, 0, 1)
            self.gen.append((self.space.from_unit(x), (x - self.mean) / self.sigma))
        self.handed = 0

    def _update(self, losses: List[float]):
        order = np.argsort(losses, kind="mergesort")[:self.mu]
        Y = np.stack([self.gen[i][1] for i in order])
        yw = (self.w[:, None] * Y).sum(0)
        self.mean = np.clip(self.mean + self.sigma * yw, 0, 1)
        D, B = np.linalg.eigh(self.C)
        Cinvsqrt = B @ np.diag(1 / np.sqrt(np.maximum(D, 1e-20))) @ B.T
        self.ps = (1 - self.cs) * self.ps + math.sqrt(self.cs * (2 - self.cs) * self.mueff) * (Cinvsqrt @ yw)
        self.generation += 1
        hsig = (np.linalg.norm(self.ps) / math.sqrt(1 - (1 - self.cs) ** (2 * self.generation))
                < (1.4 + 2 / (self.n + 1)) * self.chin)
        self.pc = (1 - self.cc) * self.pc + hsig * math.sqrt(self.cc * (2 - self.cc) * self.mueff) * yw
        rank_mu = sum(wi * np.outer(yi, yi) for wi, yi in zip(self.w, Y))
        self.C = ((1 - self.c1 - self.cmu) * self.C + self.c1 * (np.outer(self.pc, self.pc)
                  + (1 - hsig) * self.cc * (2 - self.cc) * self.C) + self.cmu * rank_mu)
        self.sigma *= math.exp((self.cs / self.damps) * (np.linalg.norm(self.ps) / self.chin - 1))
        self.sigma = float(min(max(self.sigma, 1e-4), 1.0))

    def _ask(self, history):
        if not self.gen:
            self._new_generation()
        if self.handed < self.lam:
            p = self.gen[self.handed][0]
            self.handed += 1
            return dict(p)
        # all handed out: need every result of this generation (failed -> worst)
        by_key: Dict[tuple, float] = {}
        for t in history:
            by_key[self.space.key(t["parameters"])] = self.loss(t)
        keys = [self.space.key(p) for p, _ in self.gen]
        if not all(k in by_key for k in keys):
            return WAIT
        losses = [by_key[k] if by_key[k] is not None else float("inf") for k in keys]
        self._update(losses)
        self._new_generation()
        p = self.gen[0][0]
        self.handed = 1
        return dict(p)


# ------------------------------------------------------------------------------ Hyperband
class Hyperband(Suggester):
    """Hyperband over successive-halving brackets.  Katib settings: ``resource_name`` (the
    parameter that carries the budget, e.g. epochs), ``eta`` (default 3), ``r_l`` (max
    resource R).  A bracket's rung evaluates n_i configurations with r_i resource; the top
    n_i/eta are promoted with eta x more resource; the rung's results are awaited (WAIT)."""
    name = "hyperband"

    def __init__(self, exp):
        super().__init__(exp)
        self.res_name = self.settings.get("resource_name")
        if not self.res_name or self.res_name not in self.space.names:
            raise ValueError("hyperband needs algorithmSettings resource_name naming a parameter")
        self.eta = self.setting("eta", 3.0)
        self.R = self.setting("r_l", None) or float(next(d.hi for d in self.space.dims if d.name == self.res_name))
        self.s_max = int(math.floor(math.log(self.R) / math.log(self.eta) + 1e-9))
        self.B = (self.s_max + 1) * self.R
        self.free = [d for d in self.space.dims if d.name != self.res_name]
        self.res_dim = next(d for d in self.space.dims if d.name == self.res_name)
        self.plan: List[Dict[str, str]] = []     # pending suggestions of the current rung
        self.rung: List[Dict[str, str]] = []     # all suggestions of the current rung
        self.brackets = list(range(self.s_max, -1, -1))
        self.s = None
        self.i = 0
        self.n = 0
        self.r = 0.0
        self.max_trials = int(exp.get("maxTrialCount", 10 ** 6))

    def _res(self, r: float) -> str:
        return self.res_dim.fmt(r)

    def _start_bracket(self):
        self.s = self.brackets.pop(0)
        self.n = int(math.ceil(self.B / self.R * self.eta ** self.s / (self.s + 1)))
        self.r = self.R * self.eta ** (-self.s)
        self.i = 0
        confs = [{d.name: d.sample(self.rng) for d in self.free} for _ in range(self.n)]
        self.rung = [dict(c, **{self.res_name: self._res(self.r)}) for c in confs]
        self.plan = list(self.rung)

    def _ask(self, history):
        if self.plan:
            return self.plan.pop(0)
        if self.s is not None and self.i < self.s:
            # promote the best of the finished rung
            res = {}
            for t in history:
                res[self.space.key(t["parameters"])] = self.loss(t)
            keys = [self.space.key(p) for p in self.rung]
            if not all(k in res for k in keys):
                return WAIT
            scored = sorted(((res[k] if res[k] is not None else float("inf")), j) for j, k in enumerate(keys))
            self.i += 1
            n_i = int(math.floor(self.n * self.eta ** (-self.i)))
            keep = max(1, n_i)
            r_i = self.r * self.eta ** self.i
            self.rung = [dict(self.rung[j], **{self.res_name: self._res(r_i)}) for _, j in scored[:keep]]
            self.plan = list(self.rung)
            return self.plan.pop(0)
        if not self.brackets:
            return None
        self._start_bracket()
        return self.plan.pop(0)


# ------------------------------------------------------------------------------ PBT
class PBT(Suggester):
    """Population-based training.  Each generation runs ``n_population`` members; the
    bottom ``truncation_threshold`` fraction exploits a random top member (copies its
    hyper-parameters and continues from its checkpoint) and explores (numeric values x0.8
    or x1.2, categoricals resampled with ``resample_probability``); the rest continue from
    their own checkpoint.  Trials receive ``checkpoint_dir`` (write) and
    ``parent_checkpoint_dir`` (read; empty in generation 0) as extra parameters."""
    name = "pbt"

    def __init__(self, exp, root: str = "."):
        super().__init__(exp)
        self.pop_n = int(self.setting("n_population", 8))
        self.trunc = self.setting("truncation_threshold", 0.2)
        self.resample_p = self.setting("resample_probability", 0.0)
        self.root = self.settings.get("suggestion_trial_dir") or root
        self.gen = 0
        self.members: List[Dict[str, str]] = []
        self.plan: List[Dict[str, str]] = []
        self.uid = 0

    def _ckpt(self) -> str:
        self.uid += 1
        return f"{self.root}/pbt-{self.gen}-{self.uid}"

    def _explore(self, p: Dict[str, str]) -> Dict[str, str]:
        q = dict(p)
        for d in self.space.dims:
            if d.choices is not None:
                if self.rng.random() < max(self.resample_p, 0.2 if d.categorical else 0.0):
                    q[d.name] = d.sample(self.rng)
                elif not d.categorical:
                    i = d.choices.index(q[d.name]) + self.rng.choice((-1, 1))
                    q[d.name] = d.choices[min(max(i, 0), len(d.choices) - 1)]
            elif self.resample_p and self.rng.random() < self.resample_p:
                q[d.name] = d.sample(self.rng)
            else:
                q[d.name] = d.fmt(float(q[d.name]) * self.rng.choice((0.8, 1.2)))
        return q

    def _ask(self, history):
        if self.plan:
            return self.plan.pop(0)
        if not self.members:
            for _ in range(self.pop_n):
                self.members.append(dict(self.space.sample(self.rng), checkpoint_dir=self._ckpt(),
                                         parent_checkpoint_dir=""))
            self.plan = list(self.members)
            return self.plan.pop(0)
        res = {t["parameters"].get("checkpoint_dir"): self.loss(t) for t in history}
        if not all(m["checkpoint_dir"] in res for m in self.members):
            return WAIT
        scored = sorted(((res[m["checkpoint_dir"]] if res[m["checkpoint_dir"]] is not None else float("inf")), j)
                        for j, m in enumerate(self.members))
        n_cut = max(1, int(math.ceil(self.trunc * self.pop_n)))
        top = [j for _, j in scored[:n_cut]]
        bottom = {j for _, j in scored[-n_cut:]} if len(scored) > n_cut else set()
        self.gen += 1
        nxt = []
        for j, m in enumerate(self.members):
            hp = {d.name: m[d.name] for d in self.space.dims}
            if j in bottom:
                src = self.members[self.rng.choice(top)]
                hp = self._explore({d.name: src[d.name] for d in self.space.dims})
                parent = src["checkpoint_dir"]
            else:
                parent = m["checkpoint_dir"]
            nxt.append(dict(hp, checkpoint_dir=self._ckpt(), parent_checkpoint_dir=parent))
        self.members = nxt
        self.plan = list(nxt)
        return self.plan.pop(0)


# ------------------------------------------------------------------------------ NAS
def _nas(exp: dict):
    nas = exp.get("nasConfig") or {}
    g = nas.get("graphConfig") or {}
    ops = []
    for op in nas.get("operations") or []:
        ptype = op.get("operationType")
        ps = op.get("parameters") or []
        grids = [[str(x) for x in (p.get("feasibleSpace") or {}).get("list", [])] or
                 [str(v) for v in range(int(p["feasibleSpace"]["min"]), int(p["feasibleSpace"]["max"]) + 1,
                                        int(p["feasibleSpace"].get("step", 1)))] for p in ps]
        for combo in itertools.product(*grids) if grids else [()]:
            d = {"opt_type": ptype, "opt_params": {p["name"]: v for p, v in zip(ps, combo)}}
            ops.append(d)
    return int(g.get("numLayers", 4)), g, ops


class ENAS(Suggester):
    """ENAS-style architecture search: a policy over (operation, skip connections) per
    layer, trained with REINFORCE on the trials' objective (reward = metric for maximize,
    -metric for minimize) with an exponential moving-average baseline.  Suggestions carry
    Katib's ENAS trial parameters: ``architecture`` (per layer [op, skip_0..skip_{l-1}])
    and ``nn_config`` (graph config + the operation table), both JSON."""
    name = "enas"

    def __init__(self, exp):
        self.exp = exp
        self.space = None
        self.settings = settings_of(exp)
        obj = exp.get("objective") or {}
        self.minimize = obj.get("type", "maximize") == "minimize"
        self.max_trials = int(exp.get("maxTrialCount", 10))
        seed = int(self.settings.get("random_state") or 0)
        self.rng = random.Random(seed)
        self.nrng = np.random.default_rng(seed)
        self.issued = 0
        self.L, self.graph, self.ops = _nas(exp)
        if not self.ops:
            raise ValueError("enas needs nasConfig.operations")
        self.lr = float(self.settings.get("controller_learning_rate") or 0.2)
        self.op_logits = np.zeros((self.L, len(self.ops)))
        self.skip_logits = [np.zeros(l) for l in range(self.L)]
        self.baseline = None
        self.seen = set()
        self.samples: Dict[str, list] = {}

    def loss(self, t):
        return Suggester.loss(self, t)

    def _update(self, history):
        for t in history:
            a = t["parameters"].get("architecture")
            if a is None or a in self.seen or a not in self.samples:
                continue
            self.seen.add(a)
            l = self.loss(t)
            if l is None:
                continue
            reward = -l
            self.baseline = reward if self.baseline is None else 0.8 * self.baseline + 0.2 * reward
            adv = reward - self.baseline
            arch = json.loads(a)
            for i, layer in enumerate(arch):
                p = np.exp(self.op_logits[i] - self.op_logits[i].max())
                p /= p.sum()
                g = -p
                g[layer[0]] += 1
                self.op_logits[i] += self.lr * adv * g
                for j, s in enumerate(layer[1:]):
                    q = 1 / (1 + math.exp(-self.skip_logits[i][j]))
                    self.skip_logits[i][j] += self.lr * adv * (s - q)

    def _ask(self, history):
        self._update(history)
        arch = []
        for i in range(self.L):
            p = np.exp(self.op_logits[i] - self.op_logits[i].max())
            p /= p.sum()
            op = int(self.nrng.choice(len(self.ops), p=p))
            skips = [int(self.nrng.random() < 1 / (1 + math.exp(-x))) for x in self.skip_logits[i]]
            arch.append([op] + skips)
        a = json.dumps(arch)
        self.samples[a] = arch
        cfg = {"num_layers": self.L, "input_sizes": self.graph.get("inputSizes"),
               "output_sizes": self.graph.get("outputSizes"), "embedding": {str(k): o for k, o in enumerate(self.ops)}}
        return {"architecture": a, "nn_config": json.dumps(cfg, sort_keys=True)}


class DARTS(Suggester):
    """DARTS: the differentiable search runs inside ONE trial (Katib's darts suggestion
    emits a single trial carrying the search space and settings); the trial is
    ``python -m mxtrain.workloads.nas.darts`` reading these parameters."""
    name = "darts"

    def __init__(self, exp):
        self.exp = exp
        self.space = None
        self.settings = settings_of(exp)
        self.max_trials = 1
        self.issued = 0
        self.minimize = (exp.get("objective") or {}).get("type", "maximize") == "minimize"
        self.L, self.graph, self.ops = _nas(exp)

    def _ask(self, history):
        # Katib's naming: <operationType>_<k>x<k> per filter size, bare type otherwise
        prims = sorted({o["opt_type"] + "".join(f"_{v}x{v}" for v in o["opt_params"].values())
                        for o in self.ops})
        return {"algorithm-settings": json.dumps(self.settings, sort_keys=True),
                "search-space": json.dumps(prims), "num-layers": str(self.L)}


ALGORITHMS = {
    "random": RandomSearch, "grid": GridSearch, "sobol": SobolSearch, "tpe": TPE,
    "multivariate-tpe": lambda exp: TPE(exp, multivariate=True), "bayesianoptimization": BayesOpt,
    "cmaes": CMAES, "hyperband": Hyperband, "pbt": PBT, "enas": ENAS, "darts": DARTS,
}


def make_suggester(exp: dict, root: str = ".") -> Suggester:
    alg = (exp.get("algorithm") or {}).get("algorithmName", "random")
    if alg not in ALGORITHMS:
        raise ValueError(f"algorithm {alg} not supported ({', '.join(sorted(ALGORITHMS))})")
    if alg == "pbt":
        return PBT(exp, root)
    return ALGORITHMS[alg](exp)

"""Katib search-space encoding (Experiment ``spec.parameters``).

Each parameter maps to one coordinate of the unit cube so that model-based suggestion
algorithms (TPE, GP Bayesian optimisation, CMA-ES, Sobol) work on one representation:

* ``double``       feasibleSpace min/max (optional ``step``), ``scale: log`` -> log-uniform
* ``int``          min/max (optional ``step``)
* ``discrete``     feasibleSpace.list of numbers (ordered; index coordinate)
* ``categorical``  feasibleSpace.list of strings (unordered; index coordinate)

Values handed to trials are strings, as Katib substitutes them into the trial template
(reference: charts/ml-platform/kubeflow-katib, Experiment CRD parameterSpec).
"""
from __future__ import annotations

import math
import random
from typing import Dict, List, Sequence


class Dim:
    def __init__(self, p: dict):
        self.name = p["name"]
        self.type = p.get("parameterType", "double")
        fs = p.get("feasibleSpace") or {}
        self.log = p.get("scale") == "log" or fs.get("scale") == "log"
        if self.type in ("categorical", "discrete"):
            self.choices = [str(x) for x in fs["list"]]
            if not self.choices:
                raise ValueError(f"parameter {self.name}: empty feasibleSpace.list")
            self.lo, self.hi = 0.0, float(len(self.choices) - 1)
        else:
            self.choices = None
            self.lo, self.hi = float(fs["min"]), float(fs["max"])
            if self.hi < self.lo:
                raise ValueError(f"parameter {self.name}: max < min")
            if self.log and self.lo <= 0:
                raise ValueError(f"parameter {self.name}: log scale needs min > 0")
        self.step = float(fs["step"]) if fs.get("step") not in (None, "") else None

    @property
    def categorical(self) -> bool:
        return self.type == "categorical"

    @property
    def n_choices(self) -> int:
        return len(self.choices) if self.choices is not None else 0

    # ---------------------------------------------------------------- unit <-> value
    def from_unit(self, u: float) -> str:
        u = min(max(float(u), 0.0), 1.0)
        if self.choices is not None:
            return self.choices[min(int(u * len(self.choices)), len(self.choices) - 1)]
        if self.log:
            v = math.exp(math.log(self.lo) + u * (math.log(self.hi) - math.log(self.lo)))
        else:
            v = self.lo + u * (self.hi - self.lo)
        return self.fmt(v)

    def to_unit(self, s: str) -> float:
        if self.choices is not None:
            i = self.choices.index(str(s))
            return (i + 0.5) / len(self.choices)
        v = float(s)
        if self.hi == self.lo:
            return 0.5
        if self.log:
            return (math.log(v) - math.log(self.lo)) / (math.log(self.hi) - math.log(self.lo))
        return (v - self.lo) / (self.hi - self.lo)

    def fmt(self, v: float) -> str:
        v = min(max(v, self.lo), self.hi)
        if self.step:
            v = self.lo + round((v - self.lo) / self.step) * self.step
            v = min(v, self.hi)
        if self.type == "int":
            return str(int(round(v)))
        return f"{v:.6g}"

    def grid(self) -> List[str]:
        if self.choices is not None:
            return list(self.choices)
        if self.type == "int":
            st = int(self.step or 1)
            return [str(v) for v in range(int(self.lo), int(self.hi) + 1, st)]
        step = self.step or ((self.hi - self.lo) / 4 if self.hi > self.lo else 1.0)
        out, v = [], self.lo
        while v <= self.hi + 1e-12:
            out.append(f"{v:.6g}")
            v += step
        return out

    def sample(self, r: random.Random) -> str:
        if self.choices is not None:
            return r.choice(self.choices)
        return self.from_unit(r.random())


class Space:
    def __init__(self, params: Sequence[dict]):
        self.dims = [Dim(p) for p in params]
        self.names = [d.name for d in self.dims]

    def __len__(self):
        return len(self.dims)

    def sample(self, r: random.Random) -> Dict[str, str]:
        return {d.name: d.sample(r) for d in self.dims}

    def from_unit(self, u: Sequence[float]) -> Dict[str, str]:
        return {d.name: d.from_unit(x) for d, x in zip(self.dims, u)}

    def to_unit(self, params: Dict[str, str]) -> List[float]:
        return [d.to_unit(params[d.name]) for d in self.dims]

    def key(self, params: Dict[str, str]) -> tuple:
        return tuple(str(params.get(n)) for n in self.names)

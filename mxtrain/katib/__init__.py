"""Katib-equivalent hyper-parameter / architecture search (suggestion algorithms,
metrics collectors, search space); the experiment controller is mxtrain.hpo."""
from .suggest import ALGORITHMS, WAIT, make_suggester  # noqa: F401

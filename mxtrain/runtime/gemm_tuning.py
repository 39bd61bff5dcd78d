"""Tuned GEMM selection for the library GEMMs (K12).

The plain GEMMs of the GPT/BERT steps go to hipBLASLt/rocBLAS through torch.  For each
(transpose, M, N, K, ld) of the flagship configs, PyTorch's TunableOp benchmarked every
hipBLASLt and rocBLAS solution on an MI355X and the winners are checked in under
``mxtrain/tuning/*.csv`` (validator lines pin the torch / HIP / hipBLASLt / rocBLAS
versions and gfx950; TunableOp ignores a file whose validators do not match the box).
Loading them is read-only -- no tuning happens during a run unless ``tune=True``
(``scripts/tune_gemms.sh`` regenerates the tables).

Measured on the GPT-2 345M bench (1 x MI355X, hipGraph): 19.81 -> 19.17 ms/step.
"""
from __future__ import annotations

import glob
import os
import tempfile

import torch

TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


def tuned_tables():
    return sorted(glob.glob(os.path.join(TUNING_DIR, "tunableop_*_gfx950.csv")))


def use_tuned_gemms(tune: bool = False, tables=None) -> int:
    """Enable TunableOp with the checked-in solution tables.  Returns the number of
    tables accepted (0 on CPU)."""
    if not torch.cuda.is_available():
        return 0
    import torch.cuda.tunable as tn
    tn.enable(True)
    tn.tuning_enable(bool(tune))
    # results are written back on exit: keep that out of the working directory unless tuning
    out = os.environ.get("PYTORCH_TUNABLEOP_FILENAME") or os.path.join(
        tempfile.gettempdir(), f"mxtrain_tunableop_{os.getpid()}.csv")
    tn.set_filename(out)
    n = 0
    for path in tables if tables is not None else tuned_tables():
        try:
            n += 1 if tn.read_file(path) else 0
        except Exception:
            pass
    return n

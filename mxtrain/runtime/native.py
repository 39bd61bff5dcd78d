"""ctypes binding of ``mxtrain/lib/libmxruntime.so`` (host C++ runtime helpers, built by
mxtrain.build from csrc/runtime/*.cpp).  Built on first use if absent (g++ only, no GPU
toolchain needed), so CPU-only nodes get the native path too."""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_LIB = None
_LOCK = threading.Lock()

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            from .. import build
            path = build.RUNTIME_LIB
            srcs = [os.path.join(build.CSRC, "runtime", f) for f in os.listdir(os.path.join(build.CSRC, "runtime"))]
            if not os.path.exists(path) or build._newer(srcs, path):
                build.build_runtime()
            L = ctypes.CDLL(path)
            L.mx_sample_count.argtypes = [_I64, _I64, _I32]
            L.mx_sample_count.restype = _I64
            L.mx_build_sample_idx.argtypes = [_P, _P, _I64, _I32, _I64, _P]
            L.mx_build_sample_idx.restype = ctypes.c_int
            L.mx_build_blending_indices.argtypes = [_P, _P, _P, _I32, _I64]
            L.mx_build_blending_indices.restype = None
            _LIB = L
    return _LIB


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def sample_count(num_epochs: int, tokens_per_epoch: int, seq_length: int) -> int:
    return int(lib().mx_sample_count(num_epochs, tokens_per_epoch, seq_length))


def build_sample_idx(sizes: np.ndarray, doc_idx: np.ndarray, seq_length: int, num_samples: int) -> np.ndarray:
    sizes = np.ascontiguousarray(sizes, dtype=np.int32)
    doc_idx = np.ascontiguousarray(doc_idx, dtype=np.int32)
    out = np.zeros((num_samples + 1, 2), dtype=np.int64)
    rc = lib().mx_build_sample_idx(_ptr(sizes), _ptr(doc_idx), len(doc_idx), seq_length, num_samples, _ptr(out))
    if rc != 0:
        raise RuntimeError("build_sample_idx: document stream too short for the requested samples")
    return out


def build_blending_indices(weights, size: int):
    w = np.ascontiguousarray(weights, dtype=np.float64)
    di = np.zeros(size, dtype=np.uint8)
    dsi = np.zeros(size, dtype=np.int64)
    lib().mx_build_blending_indices(_ptr(di), _ptr(dsi), _ptr(w), len(w), size)
    return di, dsi

"""hipGraph post-processing between capture and instantiation (csrc/graph.hip).

``census(g)`` counts the nodes of a captured graph by kind (kernel, memcpy, memset, ...);
``memsets_to_kernels(g)`` replaces every memset node by a fill-kernel node with the same
edges -- memset nodes replay wrong under this runtime's graph packet capture (csrc/graph.hip,
scripts/probe_graph_memsets.py).  Use with ``torch.cuda.CUDAGraph(keep_graph=True)``:

    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, ...):
        ...
    memsets_to_kernels(g)      # before instantiate() / the first replay
    g.instantiate()
"""
from __future__ import annotations

import ctypes
from typing import Dict

NODE_TYPES = ("kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event", "event_record",
              "ext_sem_signal", "ext_sem_wait", "mem_alloc", "mem_free", "memcpy_from_symbol",
              "memcpy_to_symbol", "batch_mem_op")


def census(g) -> Dict[str, int]:
    from ..ops import _lib
    counts = (ctypes.c_int * len(NODE_TYPES))()
    n = _lib._fn("mx_graph_census")(int(g.raw_cuda_graph()), counts, len(NODE_TYPES))
    if n < 0:
        raise RuntimeError("hipGraph node census failed")
    out = {name: int(c) for name, c in zip(NODE_TYPES, counts) if c}
    out["total"] = int(n)
    return out


def memsets_to_kernels(g) -> int:
    """Replace the captured graph's memset nodes by fill-kernel nodes; returns how many."""
    from ..ops import _lib
    n = _lib._fn("mx_graph_memsets_to_kernels")(int(g.raw_cuda_graph()))
    if n < 0:
        raise RuntimeError(f"rewriting the graph's memset nodes failed ({n})")
    return int(n)

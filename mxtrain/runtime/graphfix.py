"""hipGraph post-processing between capture and instantiation (csrc/graph.hip).

``snapshot_host_copies(g)`` rewrites every memcpy node of a captured graph whose source is
host memory into a device-to-device copy from a device snapshot of those bytes, taken now
(see the top of csrc/graph.hip for why).  Use with ``torch.cuda.CUDAGraph(keep_graph=True)``:

    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, ...):
        ...
    fix = snapshot_host_copies(g)      # before the first replay / instantiate()
    g.instantiate()
    ...
    fix.release()                      # when the graph is dropped
"""
from __future__ import annotations

import ctypes
from typing import Dict, List

NODE_TYPES = ("kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event", "event_record",
              "ext_sem_signal", "ext_sem_wait", "mem_alloc", "mem_free", "memcpy_from_symbol",
              "memcpy_to_symbol", "batch_mem_op")


def _raw(g) -> int:
    return int(g.raw_cuda_graph())


def census(g) -> Dict[str, int]:
    from ..ops import _lib
    counts = (ctypes.c_int * len(NODE_TYPES))()
    n = _lib._fn("mx_graph_census")(_raw(g), counts, len(NODE_TYPES))
    if n < 0:
        raise RuntimeError("hipGraph node census failed")
    out = {name: int(c) for name, c in zip(NODE_TYPES, counts) if c}
    out["total"] = int(n)
    return out


def memcpy_nodes(g, max_rows: int = 4096) -> List[dict]:
    from ..ops import _lib
    rows = (ctypes.c_int64 * (5 * max_rows))()
    n = _lib._fn("mx_graph_memcpy_nodes")(_raw(g), rows, max_rows)
    if n < 0:
        raise RuntimeError(f"reading the graph's memcpy nodes failed ({n})")
    mt = {1: "host", 2: "device", -1: "unreadable"}
    return [{"src": rows[5 * i], "dst": rows[5 * i + 1], "bytes": rows[5 * i + 2], "src_mem": mt.get(rows[5 * i + 3]),
             "dst_mem": mt.get(rows[5 * i + 4])} for i in range(min(n, max_rows))]


class HostCopySnapshots:
    """Device buffers backing the rewritten nodes; they must outlive every replay."""

    def __init__(self, bufs: List[int]):
        self.bufs = bufs

    def __len__(self) -> int:
        return len(self.bufs)

    def release(self) -> None:
        if self.bufs:
            from ..ops import _lib
            arr = (ctypes.c_void_p * len(self.bufs))(*self.bufs)
            _lib._fn("mx_graph_free")(arr, len(self.bufs))
            self.bufs = []


def snapshot_host_copies(g, max_nodes: int = 4096) -> HostCopySnapshots:
    from ..ops import _lib
    arr = (ctypes.c_void_p * max_nodes)()
    n = _lib._fn("mx_graph_snapshot_h2d")(_raw(g), arr, max_nodes)
    if n < 0:
        raise RuntimeError(f"rewriting the graph's host-sourced copies failed ({n})")
    return HostCopySnapshots([int(arr[i]) for i in range(n)])

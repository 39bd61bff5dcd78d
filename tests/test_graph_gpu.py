"""hipGraph post-processing (csrc/graph.hip, mxtrain.runtime.graphfix) on the GPU.

With the runtime's graph packet capture (the default of this HIP runtime), a graph holding
a host-to-device copy node replays later [memset, accumulate] rounds out of order
(scripts/probe_graph_nodes.py).  These tests capture such a graph, rewrite its host-sourced
copies into device snapshots, and check every round of the replay exactly.  No kernel here
indexes memory with data, so a misordered node cannot fault.
"""
import ctypes
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _hip():
    return ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


def _capture(hip, rounds, n, with_h2d):
    acc = torch.zeros(n, dtype=torch.int32, device="cuda")
    out = torch.zeros(rounds, n, dtype=torch.int32, device="cuda")
    dst = torch.zeros(n, dtype=torch.int32, device="cuda")
    host = (ctypes.c_int * n)(*range(n))          # pageable host memory

    def body(stream):
        if with_h2d:
            assert hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.cast(host, ctypes.c_void_p),
                                      ctypes.c_size_t(4 * n), 1, ctypes.c_void_p(stream)) == 0
        for r in range(rounds):
            assert hip.hipMemsetAsync(ctypes.c_void_p(acc.data_ptr()), 0, ctypes.c_size_t(4 * n),
                                      ctypes.c_void_p(stream)) == 0
            acc.add_(1)
            acc.add_(dst[:1])     # reads the copied data (0 from the copy) into every round
            out[r].copy_(acc)

    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.stream(s):
        body(s.cuda_stream)        # warm-up outside the capture
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        body(s.cuda_stream)
    return g, acc, out, dst, host


@pytest.mark.parametrize("with_h2d", [False, True])
def test_graph_memset_rounds_exact_after_host_copy_snapshot(with_h2d):
    from mxtrain.runtime import graphfix
    hip = _hip()
    rounds, n = 64, 4096
    g, acc, out, dst, host = _capture(hip, rounds, n, with_h2d)
    census = graphfix.census(g)
    assert census["memset"] >= rounds
    fix = graphfix.snapshot_host_copies(g)
    assert len(fix) == (1 if with_h2d else 0)
    if with_h2d:
        mc = graphfix.memcpy_nodes(g)
        assert all(m["src_mem"] == "device" for m in mc)   # every host-sourced copy rewritten
        for i in range(n):                                # the replay must not see this
            host[i] = 99
    g.instantiate()
    for _ in range(3):
        out.fill_(-1)
        acc.fill_(-1)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, torch.ones_like(out)), (out != 1).any(1).nonzero().flatten().tolist()[:8]
        assert torch.equal(dst.cpu(), torch.arange(n, dtype=torch.int32)) or not with_h2d
    del g
    torch.cuda.synchronize()
    fix.release()

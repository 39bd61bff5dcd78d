"""hipGraph post-processing (csrc/graph.hip, mxtrain.runtime.graphfix) under the runtime's
graph packet capture (this runtime's default): memset nodes replay wrong there
(scripts/probe_graph_memsets.py, profiles/r3_s4/), so captured graphs have them replaced by
fill-kernel nodes; with that, rounds of [memset, accumulate, copy, snapshot] replay exactly,
every round, every replay.  No kernel here indexes memory with data, so a misordered node
cannot fault.
"""
import ctypes
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbytes", [4096 * 4, 4, 12, 1022])
def test_graph_memset_nodes_as_kernels_replay_exactly(nbytes):
    from mxtrain.runtime import graphfix
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    rounds, n = 64, 4096
    nb = nbytes
    acc = torch.zeros(n, dtype=torch.int32, device="cuda")
    out = torch.zeros(rounds, n, dtype=torch.int32, device="cuda")
    src = torch.arange(n, dtype=torch.int32, device="cuda")
    cpy = torch.zeros(n, dtype=torch.int32, device="cuda")

    def body(stream):
        for r in range(rounds):
            acc.fill_(5)
            assert hip.hipMemsetAsync(ctypes.c_void_p(acc.data_ptr()), 0, ctypes.c_size_t(nb),
                                      ctypes.c_void_p(stream)) == 0
            acc.add_(1)
            acc.add_(1)
            assert hip.hipMemcpyAsync(ctypes.c_void_p(cpy.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                      ctypes.c_size_t(4 * n), 3, ctypes.c_void_p(stream)) == 0
            acc.add_(cpy[:1])      # + 0: the device-to-device copy is ordered before it
            out[r].copy_(acc)

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        body(s.cuda_stream)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=s):
        body(s.cuda_stream)
    c = graphfix.census(g)
    assert c["memset"] == rounds and c["memcpy"] >= rounds and c["kernel"] >= 3 * rounds, c
    assert graphfix.memsets_to_kernels(g) == rounds
    c2 = graphfix.census(g)
    assert "memset" not in c2 and c2["kernel"] == c["kernel"] + rounds and c2["total"] == c["total"], c2
    g.instantiate()
    # reference: the same rounds run eagerly
    out.fill_(-1)
    body(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = out.clone()
    nz = nb // 4                       # whole ints zeroed; a partial int keeps its upper bytes
    assert (ref[:, :nz] == 2).all() and (ref[:, (nb + 3) // 4:] == 7).all()
    for _ in range(3):
        out.fill_(-1)
        acc.fill_(-1)
        cpy.fill_(-1)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        bad = (out != ref).any(1).nonzero().flatten().tolist()
        assert not bad, f"rounds {bad[:8]} wrong"

"""xGMI preflight (mxtrain/parallel/preflight.py) on the box's one MI355X: two job ranks
(plain host processes, no GPU touched) each start their throwaway child; the children
share the GPU (RCCL's side emulated on gloo), run the IPC handle exchange, the
registered-buffer self-test, the autotune against the reference collective and the p2p
round trip, and both ranks must read the same positive verdict.  A child that fails on one
rank must turn the kernels off on both (the CPU test covers the gloo stand-in;
here the real kernels run)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, env, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", MXTRAIN_XGMI="auto", MXTRAIN_PREFLIGHT_EMU="1", **env)
    os.environ.pop("MXTRAIN_XGMI_PREFLIGHT_DONE", None)
    from mxtrain.parallel import preflight
    v = preflight.run_preflight(world, rank, timeout_s=90)
    q.put((rank, v, os.environ.get("MXTRAIN_XGMI")))


@pytest.mark.parametrize("fail", [None, 1])
def test_preflight_children_on_gpu(fail):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    env = {} if fail is None else {"MXTRAIN_PREFLIGHT_FAIL_RANK": str(fail)}
    ps = [ctx.Process(target=_rank, args=(r, 2, port, env, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict((r, (v, m)) for r, v, m in (q.get(timeout=150) for _ in ps))
    for p in ps:
        p.join(30)
    v0, v1 = out[0][0], out[1][0]
    assert v0["ok"] == v1["ok"], (v0, v1)
    if fail is None:
        assert v0["ok"], v0
        assert v0.get("p2p_ok") and v0.get("direct_ok"), v0
        assert out[0][1] == out[1][1] == "auto"
    else:
        assert not v0["ok"] and "rank 1" in v0["reason"], v0
        assert out[0][1] == out[1][1] == "0"

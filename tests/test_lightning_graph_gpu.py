"""The Lightning-style trainer's hipGraph step (mxtrain/raylike/lightning.py): after three
eager steps the whole training step -- bf16-autocast forward of a BatchNorm ResNet-50,
backward, SGD-Nesterov with a per-step LambdaLR rate read from device scalars -- is
captured once and replayed.  Against the same run with the graph off: every step's loss and
the final weights stay within 5 % of the run's update norm (the captured SGD computes
p -= lr * d in two roundings where torch's fused add uses one, and bf16 training carries
that forward), and the BatchNorm step counters advance identically."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graph: bool, steps: int = 8, batch: int = 16, size: int = 224):
    from mxtrain.raylike import lightning as L
    from mxtrain.workloads.ray.train_resnet50 import ResNet50Module
    torch.manual_seed(0)
    model = ResNet50Module(0.05, total=steps)
    g = torch.Generator().manual_seed(1)
    xs = torch.randint(0, 256, (steps, batch, 3, size, size), dtype=torch.uint8, generator=g)
    ys = torch.randint(0, 1000, (steps, batch), generator=g)
    m = ResNet50Module(0.05, total=steps)
    m.load_state_dict(model.state_dict())
    tr = L.Trainer(max_epochs=1, precision="bf16-mixed", hipgraph=graph, enable_progress_bar=False)
    tr.fit(m, train_dataloaders=[(xs[i], ys[i]) for i in range(steps)])
    torch.cuda.synchronize()
    return tr, m


def test_graphed_resnet50_step_matches_eager():
    tr_e, me = _run(False)
    tr_g, mg = _run(True)
    assert tr_g.graph_info.get("captured_at_step") == 3, tr_g.graph_info
    assert tr_g.graph_info["nodes"]["kernel"] > 100, tr_g.graph_info
    assert "error" not in tr_e.graph_info
    se, sg, s0 = me.state_dict(), mg.state_dict(), _init_state()
    num = den = 0.0
    for k, v in se.items():
        a, b = v.float(), sg[k].float()
        if "num_batches_tracked" in k:
            assert torch.equal(a, b), k
            continue
        num += float(((a - b) ** 2).sum())
        den += float(((a - s0[k].float().to(a.device)) ** 2).sum())
    # the graphed SGD rounds p - lr d in two steps where torch's fused add rounds once; bf16
    # training carries such differences forward, so judge against the total update size
    drift = (num / den) ** 0.5
    print(f"[lightning-graph] drift vs eager: {drift:.4f} of the update norm")
    assert drift < 0.05, drift
    le, lg = tr_e.callback_metrics["train_loss"], tr_g.callback_metrics["train_loss"]
    assert abs(le - lg) <= 2e-3 * abs(le), (le, lg)


def _init_state():
    from mxtrain.workloads.ray.train_resnet50 import ResNet50Module
    torch.manual_seed(0)
    return ResNet50Module(0.05, total=8).state_dict()


def test_sgd_multi_matches_torch_sgd():
    """raylike/lightning.py sgd_step_device_lr on the one-launch HIP update (csrc/optim.hip
    mx_sgd_multi: weight decay, momentum, Nesterov, LR from a device scalar) against
    torch.optim.SGD over three steps: channels_last conv weights, vectors, a matrix."""
    import torch
    from mxtrain.raylike.lightning import sgd_step_device_lr
    torch.manual_seed(0)
    shapes = [(64, 32, 3, 3), (256,), (100, 48), (128, 64, 1, 1)]
    mk = lambda: [torch.nn.Parameter(torch.randn(s, device="cuda").contiguous(  # noqa: E731
        memory_format=torch.channels_last if len(s) == 4 else torch.contiguous_format)) for s in shapes]
    a, b = mk(), mk()
    for x, y in zip(a, b):
        y.data.copy_(x.data)
    kw = dict(lr=0.05, momentum=0.9, nesterov=True, weight_decay=1e-3)
    oa, ob = torch.optim.SGD(a, **kw), torch.optim.SGD(b, **kw)
    lrs = [torch.tensor(0.05, device="cuda")]
    for _ in range(3):
        gs = [torch.randn(s, device="cuda") for s in shapes]
        for x, y, g in zip(a, b, gs):
            x.grad = g.clone().contiguous(memory_format=torch.channels_last if g.dim() == 4 else torch.contiguous_format)
            y.grad = x.grad.clone()
        oa.step()
        sgd_step_device_lr(ob, lrs)
    for x, y in zip(a, b):
        torch.testing.assert_close(y, x, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(ob.state[y]["momentum_buffer"], oa.state[x]["momentum_buffer"], rtol=1e-6, atol=1e-6)

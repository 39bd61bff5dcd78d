"""FlatMaster (models/compute_weights.py): flat fp32 master / grads / momentum with
persistent compute copies must reproduce torch.optim.SGD (momentum, per-group weight decay)
+ torch.nn.utils.clip_grad_norm_ on a model whose convs carry folded per-channel scales.
CPU path (torch ops); the GPU path runs the same contract through csrc/multitensor.hip
(tests/test_maskrcnn_gpu.py::test_flat_master_gpu_matches_cpu)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mxtrain.models.compute_weights import FlatMaster, cw


class Tiny(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3, padding=1)
        self.conv2 = nn.Conv2d(8, 4, 1)
        self.fc = nn.Linear(4 * 6 * 6, 5)
        self.frozen = nn.Parameter(torch.randn(5), requires_grad=False)
        self.register_buffer("s", torch.rand(8) + 0.5)
        self._specs = None

    def compute_weight_specs(self):
        if self._specs is None:
            full = self.s[:, None, None, None].expand_as(self.conv.weight).contiguous()
            self._specs = [(self.conv.weight, full)] + [(p, None) for n, p in self.named_parameters()
                                                        if p.requires_grad and n != "conv.weight"]
        return self._specs

    def forward(self, x, folded_ref=False):
        dt = x.dtype
        w = cw(self.conv.weight, dt) if not folded_ref else self.conv.weight * self.s[:, None, None, None]
        y = F.relu(F.conv2d(x, w, cw(self.conv.bias, dt) if not folded_ref else self.conv.bias, padding=1))
        y = F.conv2d(y, cw(self.conv2.weight, dt) if not folded_ref else self.conv2.weight,
                     cw(self.conv2.bias, dt) if not folded_ref else self.conv2.bias)
        y = y.flatten(1)
        fw = cw(self.fc.weight, dt) if not folded_ref else self.fc.weight
        fb = cw(self.fc.bias, dt) if not folded_ref else self.fc.bias
        return (F.linear(y, fw, fb) + self.frozen).pow(2).mean()


def _opt(m):
    decay = [p for p in m.parameters() if p.requires_grad and p.ndim > 1]
    no_decay = [p for p in m.parameters() if p.requires_grad and p.ndim <= 1]
    return torch.optim.SGD([{"params": decay, "weight_decay": 1e-2}, {"params": no_decay, "weight_decay": 0.0}],
                           lr=0.05, momentum=0.9)


@pytest.mark.parametrize("clip", [0.0, 0.05])
def test_flat_master_matches_torch_sgd(clip):
    torch.manual_seed(0)
    ref = Tiny()
    mod = copy.deepcopy(ref)
    opt_r, opt_m = _opt(ref), _opt(mod)
    fm = FlatMaster(mod, opt_m, clip, dt=torch.float32)
    xs = [torch.randn(2, 3, 6, 6) for _ in range(4)]
    for step, x in enumerate(xs):
        lr = 0.05 * (step + 1)
        for g in opt_r.param_groups:
            g["lr"] = lr
        opt_r.zero_grad(set_to_none=True)
        ref(x, folded_ref=True).backward()
        if clip > 0:
            torch.nn.utils.clip_grad_norm_([p for p in ref.parameters() if p.requires_grad], clip)
        opt_r.step()
        opt_m.zero_grad(set_to_none=True)
        with fm.compute_weights():
            loss = mod(x)
        loss.backward()
        fm.step(lr)
    for (n, a), b in zip(ref.named_parameters(), mod.parameters()):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6, msg=n)
    # the SGD state stays in the optimizer (checkpoints unchanged) and aliases the flat buffer
    sd = opt_m.state_dict()
    bufs_r = [opt_r.state[p]["momentum_buffer"] for p in opt_r.param_groups[0]["params"]]
    bufs_m = [sd["state"][i]["momentum_buffer"] for i in range(len(bufs_r))]
    for a, b in zip(bufs_r, bufs_m):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    p0 = opt_m.param_groups[0]["params"][0]
    assert opt_m.state[p0]["momentum_buffer"].data_ptr() == fm.M.data_ptr() + 4 * fm.offs[0]


def test_flat_master_recasts_after_param_write_and_rebinds_state():
    torch.manual_seed(1)
    mod = Tiny()
    opt = _opt(mod)
    fm = FlatMaster(mod, opt, 0.0, dt=torch.float32)
    fm.ensure_fresh()
    with torch.no_grad():
        mod.fc.weight.add_(1.0)          # e.g. a checkpoint load: bumps the version
    fm.ensure_fresh()
    o = [id(p) for p in fm.params].index(id(mod.fc.weight))
    torch.testing.assert_close(fm.compute_views()[o], mod.fc.weight.detach())
    # a loaded optimizer state is copied into the flat momentum buffer
    sd = opt.state_dict()
    for st in sd["state"].values():
        st["momentum_buffer"] = torch.full_like(st["momentum_buffer"], 0.5)
    for i, p in enumerate(fm.params):
        sd["state"].setdefault(i, {"momentum_buffer": torch.full_like(p, 0.5)})
    opt.load_state_dict(sd)
    fm.rebind_state()
    assert torch.all(fm.M[:fm.sizes[0]] == 0.5)
    assert opt.state[fm.params[0]]["momentum_buffer"].data_ptr() == fm.M.data_ptr()

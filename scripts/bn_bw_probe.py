"""Achieved HBM bandwidth of the trainable-BN kernels at the ResNet-50 res2 output shape
(batch 256, 56 x 56, 256 channels, bf16 NHWC): forward (statistics from a conv epilogue are
not used here: bn_stats + finalize + apply) and backward (stats + finalize + apply), timed
with events; bytes = the tensors each pass must move once."""
import torch

from mxtrain.ops.batchnorm import bn_act

N, C, H, W = 256, 256, 56, 56
cl = torch.channels_last
x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
r = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
dy = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
bn = torch.nn.BatchNorm2d(C).cuda()
nbytes = x.numel() * 2


def run(k=10):
    xa = x.clone().requires_grad_(True)
    ra = r.clone().requires_grad_(True)
    s, m, e = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    tf = tb = 0.0
    for i in range(k + 3):
        s.record()
        y = bn_act(xa, bn, ra, True)
        m.record()
        y.backward(dy)
        e.record()
        torch.cuda.synchronize()
        if i >= 3:
            tf += s.elapsed_time(m)
            tb += m.elapsed_time(e)
        xa.grad = ra.grad = None
    return tf / k * 1e3, tb / k * 1e3


tf, tb = run()
# forward: stats reads x, apply reads x + res and writes y (4 tensor passes)
# backward: stats reads dy, y, x; apply reads dy, y, x and writes dx, dres (8 passes)
print(f"tensor {nbytes / 1e6:.0f} MB  fwd {tf:.1f} us = {4 * nbytes / tf / 1e6:.2f} TB/s (4 passes)  "
      f"bwd {tb:.1f} us = {8 * nbytes / tb / 1e6:.2f} TB/s (8 passes)", flush=True)

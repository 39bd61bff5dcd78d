import sys, torch
sys.path.insert(0, "/root/repo")
from mxtrain.ops import stem as S
from mxtrain.ops import _lib as L
torch.manual_seed(0)
mean, std = (123.675, 116.28, 103.53), (58.395, 57.12, 57.375)
for (N, H, W) in [(1, 101, 133), (1, 100, 132), (1, 101, 132), (1, 100, 133), (2, 96, 160)]:
    img = torch.randint(0, 256, (N, 3, H, W), dtype=torch.uint8, device="cuda")
    wf = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).to(torch.bfloat16)
    bf = (torch.randn(64, device="cuda") * 0.1).to(torch.bfloat16)
    for gsz in (512, 1 << 30):
        L._fn("mx_stem_grid")(gsz)
        y = S.stem_pool(img, wf, bf, mean, std).float()
        ref = S.stem_pool_ref(img, wf, bf, mean, std).float()
        d = (y - ref).abs().amax(1)   # [N, PH, PW]
        bad = (d > 0.1).nonzero()
        print(N, H, W, "grid", gsz, "max err", d.max().item(), "bad px", bad.shape[0], bad[:6].tolist(), "PH,PW", tuple(y.shape[2:]), flush=True)

#!/usr/bin/env python3
"""Which part of the ResNet-50 (BatchNorm, bf16 autocast) training step breaks a hipGraph
capture: MODE=fwd | fwdbwd | full, STREAM=side (explicit stream + eager warm-up on it,
keep_graph + memset rewrite) or default (torch.cuda.graph's own stream).  One mode per
process (a failure can be a segfault)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mode = os.environ.get("MODE", "full")
    explicit = os.environ.get("STREAM", "side") == "side"
    from mxtrain.raylike.lightning import sgd_step_device_lr
    from mxtrain.workloads.ray.train_resnet50 import ResNet50Module
    import torch.nn.functional as F
    dev = torch.device("cuda")
    m = ResNet50Module(0.05).to(dev)
    opt = m.configure_optimizers()["optimizer"]
    x = torch.randint(0, 256, (int(os.environ.get("BATCH", "32")), 3, 224, 224), dtype=torch.uint8, device=dev)
    y = torch.randint(0, 1000, (x.shape[0],), device=dev)
    lrs = [torch.tensor(0.01, device=dev) for _ in opt.param_groups]

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x).float(), y, label_smoothing=0.1)
        if mode == "fwd":
            return loss
        loss.backward()
        if mode == "full":
            sgd_step_device_lr(opt, lrs)
        return loss

    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        step()
    torch.cuda.synchronize()
    print(f"eager ok ({mode}, stream {'side' if explicit else 'default'})", flush=True)
    opt.zero_grad(set_to_none=True)
    if explicit:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
            opt.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                loss = step()
        from mxtrain.runtime import graphfix
        print("census", graphfix.census(g), "memsets->kernels", graphfix.memsets_to_kernels(g), flush=True)
        g.instantiate()
        torch.cuda.current_stream().wait_stream(s)
    else:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            loss = step()
    print("captured", flush=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print("replayed ok, loss", float(loss), flush=True)


if __name__ == "__main__":
    main()

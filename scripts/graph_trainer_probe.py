#!/usr/bin/env python3
"""Lightning-style Trainer hipGraph mode on ResNet-50: FIRST=eager runs an eager fit
before the graphed one in the same process (as tests/test_lightning_graph_gpu.py);
FIRST=none runs only the graphed fit.  SIZE / BATCH / STEPS shape the synthetic batches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def fit(graph, steps, batch, size):
    from mxtrain.raylike import lightning as L
    from mxtrain.workloads.ray.train_resnet50 import ResNet50Module
    torch.manual_seed(0)
    m = ResNet50Module(0.05, total=steps)
    g = torch.Generator().manual_seed(1)
    data = [(torch.randint(0, 256, (batch, 3, size, size), dtype=torch.uint8, generator=g),
             torch.randint(0, 1000, (batch,), generator=g)) for _ in range(steps)]
    tr = L.Trainer(max_epochs=1, precision="bf16-mixed", hipgraph=graph, enable_progress_bar=False)
    print(f"fit graph={graph}", flush=True)
    tr.fit(m, train_dataloaders=data)
    torch.cuda.synchronize()
    print("done", tr.graph_info, tr.callback_metrics, flush=True)


if __name__ == "__main__":
    steps, batch, size = (int(os.environ.get(k, d)) for k, d in (("STEPS", "8"), ("BATCH", "16"), ("SIZE", "224")))
    if os.environ.get("FIRST", "none") == "eager":
        fit(False, steps, batch, size)
    fit(True, steps, batch, size)

"""ResNet-50 image classification with the Ray Train + Lightning structure of the
reference's raytrain workloads -- BASELINE config 5 ("Ray Train PyTorch Lightning
ResNet-50 N workers, synthetic ImageNet").

    python train_resnet50.py [--num-workers N] [--batch-size 256] [--epochs 1] [--steps-per-epoch 100]

The driver builds a TorchTrainer (mxtrain.raylike) over N GPU workers (default: the
RayJob worker group size); each worker runs a Lightning-style loop (BatchNorm ResNet-50,
channels_last bf16 autocast, MIOpen NHWC convs, SGD-Nesterov, label smoothing) on a
synthetic ImageNet stream (224x224 RGB, 1000 classes) and reports samples/s + loss each
epoch through ray.train.report semantics.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mxtrain.raylike import lightning as L  # noqa: E402
from mxtrain.raylike import train  # noqa: E402
from mxtrain.raylike.train import RunConfig, ScalingConfig  # noqa: E402
from mxtrain.raylike.train.torch import TorchTrainer, prepare_data_loader  # noqa: E402


class SyntheticImageNet(torch.utils.data.Dataset):
    """A fixed pool of random images (the stream cycles through it) so data loading is
    cheap and deterministic; labels are uniform over 1000 classes."""

    def __init__(self, length: int, pool: int = 256, size: int = 224, classes: int = 1000, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.images = torch.randint(0, 256, (pool, 3, size, size), dtype=torch.uint8, generator=g)
        self.labels = torch.randint(0, classes, (length,), generator=g)
        self.length = length

    def __len__(self):
        return self.length

    def __getitem__(self, i):
        return self.images[i % len(self.images)], self.labels[i]


class ResNet50Module(L.LightningModule):
    def __init__(self, lr: float, weight_decay: float = 5e-5, warmup: int = 50, total: int = 1000):
        super().__init__()
        from mxtrain.models.resnet import resnet50
        self.net = resnet50(norm="bn", num_classes=1000).to(memory_format=torch.channels_last)
        self.lr, self.wd, self.warmup, self.total = lr, weight_decay, warmup, total
        # device-resident normalisation constants (no host copies inside the step: capturable)
        self.register_buffer("mean", torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1) * 255, persistent=False)
        self.register_buffer("std", torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1) * 255, persistent=False)

    MEAN = (0.485 * 255, 0.456 * 255, 0.406 * 255)
    STD = (0.229 * 255, 0.224 * 255, 0.225 * 255)

    def forward(self, x):
        if (x.is_cuda and x.dtype == torch.uint8 and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            # uint8 NCHW -> normalised bf16 NHWC in one kernel (the autocast conv input)
            from mxtrain.ops.vision import normalize_u8_nhwc
            return self.net(normalize_u8_nhwc(x, self.MEAN, self.STD))
        x = (x.float() - self.mean) / self.std
        return self.net(x.contiguous(memory_format=torch.channels_last))

    def training_step(self, batch, idx):
        x, y = batch
        logits = self(x)
        loss = F.cross_entropy(logits.float(), y, label_smoothing=0.1)
        self.log("loss", loss)
        return loss

    def validation_step(self, batch, idx):
        x, y = batch
        acc = (self(x).argmax(-1) == y).float().mean()
        self.log("val_acc", acc, sync_dist=True)

    def configure_optimizers(self):
        decay = [p for n, p in self.named_parameters() if p.ndim > 1]
        no_decay = [p for n, p in self.named_parameters() if p.ndim <= 1]
        opt = torch.optim.SGD([{"params": decay, "weight_decay": self.wd}, {"params": no_decay, "weight_decay": 0}],
                              lr=self.lr, momentum=0.9, nesterov=True)
        import math

        def f(step):
            if step < self.warmup:
                return (step + 1) / self.warmup
            return 0.5 * (1 + math.cos(math.pi * min(1.0, (step - self.warmup) / max(1, self.total - self.warmup))))
        return {"optimizer": opt, "lr_scheduler": torch.optim.lr_scheduler.LambdaLR(opt, f)}


def train_loop_per_worker(cfg):
    ctx = train.get_context()
    bs = cfg["batch_size"]
    steps = cfg["steps_per_epoch"]
    ds = SyntheticImageNet(bs * steps * ctx.get_world_size(), seed=cfg.get("seed", 0), size=cfg.get("image_size", 224))
    dl = torch.utils.data.DataLoader(ds, batch_size=bs, shuffle=True, num_workers=cfg.get("num_workers", 4),
                                     drop_last=True, persistent_workers=cfg.get("num_workers", 4) > 0)
    dl = prepare_data_loader(dl)
    lr = cfg["lr"] * bs * ctx.get_world_size() / 256
    model = ResNet50Module(lr, total=steps * cfg["epochs"])
    trainer = L.Trainer(max_epochs=cfg["epochs"], precision="bf16-mixed", devices="auto", accelerator="auto",
                        strategy=L.RayDDPStrategy(), plugins=[L.RayLightningEnvironment()],
                        callbacks=[L.RayTrainReportCallback()], log_every_n_steps=cfg.get("log_every", 20),
                        enable_progress_bar=True, limit_train_batches=steps)
    trainer = L.prepare_trainer(trainer)
    trainer.fit(model, train_dataloaders=dl)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-workers", type=int, default=int(os.environ.get("MXTRAIN_RAY_NUM_WORKERS", "1")))
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--steps-per-epoch", type=int, default=100)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--loader-workers", type=int, default=4)
    ap.add_argument("--image-size", type=int, default=224, help="synthetic image side (tests: small)")
    ap.add_argument("--storage-path", default=os.path.join(os.environ.get("HOME", "."), "ray_results"))
    ap.add_argument("--name", default="resnet50")
    ap.add_argument("--result-json", default=None)
    a = ap.parse_args(argv)
    use_gpu = not a.cpu and torch.cuda.is_available() and os.environ.get("MXTRAIN_CPU_ONLY") != "1"
    trainer = TorchTrainer(train_loop_per_worker,
                           train_loop_config={"batch_size": a.batch_size, "epochs": a.epochs,
                                              "steps_per_epoch": a.steps_per_epoch, "lr": a.lr,
                                              "num_workers": a.loader_workers, "image_size": a.image_size},
                           scaling_config=ScalingConfig(num_workers=a.num_workers, use_gpu=use_gpu),
                           run_config=RunConfig(name=a.name, storage_path=a.storage_path))
    result = trainer.fit()
    print("Result:", json.dumps(result.metrics), flush=True)
    if a.result_json:
        rec = {"metric": "Ray Train ResNet-50 images/sec", "value": result.metrics.get("samples_per_sec"),
               "n_gpus": a.num_workers if use_gpu else 0, "batch_per_worker": a.batch_size, "checkpoint":
               result.checkpoint.path if result.checkpoint else None}
        with open(a.result_json, "a") as f:
            f.write(json.dumps(rec) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())

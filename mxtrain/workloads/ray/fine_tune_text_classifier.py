"""BERT text-classifier fine-tuning with Ray Train + Lightning -- the workload of the
reference's Ray example (kuberay sample `fine-tune-pytorch-text-classifier.py`,
examples/ray/lightning-bert/fine-tune.yaml:34-50).

The driver starts a TorchTrainer worker group (mxtrain.raylike, one rank per MI355X of
the RayJob worker group); each worker fine-tunes mxtrain's HIP BERT
(`bert-base-cased` shapes, random init) on an offline sentence-pair classification set
with a Lightning-style module (AdamW, linear schedule, bf16), reporting train loss,
validation accuracy and samples/s per epoch with a checkpoint.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))

import torch  # noqa: E402

from mxtrain.raylike import lightning as L  # noqa: E402
from mxtrain.raylike import train  # noqa: E402
from mxtrain.raylike.train import CheckpointConfig, RunConfig, ScalingConfig  # noqa: E402
from mxtrain.raylike.train.torch import TorchTrainer, prepare_data_loader  # noqa: E402


class SentimentModel(L.LightningModule):
    def __init__(self, model_name: str, lr: float, total_steps: int, vocab_size: int):
        super().__init__()
        from mxtrain.models.bert import BERT_CONFIGS, BertConfig, BertForSequenceClassification
        cfg = BertConfig(**BERT_CONFIGS[model_name])
        cfg.vocab_size = max(cfg.vocab_size, vocab_size)
        self.model = BertForSequenceClassification(cfg)
        self.lr, self.total = lr, total_steps

    def training_step(self, batch, idx):
        out = self.model(batch["input_ids"], batch["attention_mask"], batch["token_type_ids"], batch["labels"])
        self.log("train_loss", out["loss"])
        return out["loss"]

    def validation_step(self, batch, idx):
        logits = self.model(batch["input_ids"], batch["attention_mask"], batch["token_type_ids"])["logits"]
        self.log("val_accuracy", (logits.argmax(-1) == batch["labels"]).float().mean(), sync_dist=True)

    def configure_optimizers(self):
        opt = torch.optim.AdamW(self.parameters(), lr=self.lr, fused=torch.cuda.is_available() and
                                os.environ.get("MXTRAIN_CPU_ONLY") != "1")
        sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: max(0.0, 1 - s / max(1, self.total)))
        return {"optimizer": opt, "lr_scheduler": sched}


def train_func(cfg):
    from mxtrain.data.glue import bert_tokenizer, collate, mrpc_splits
    sizes = {"train": cfg["train_size"], "validation": cfg["eval_size"]}
    sp = mrpc_splits(seed=0, sizes=sizes)
    tok = bert_tokenizer(os.path.join(cfg["cache"], f"{cfg['model']}-wordpiece"))

    def encode(rows):
        enc = tok([r["sentence1"] for r in rows], [r["sentence2"] for r in rows], truncation=True, max_length=128)
        return [{"input_ids": enc["input_ids"][i], "token_type_ids": enc["token_type_ids"][i],
                 "attention_mask": enc["attention_mask"][i], "labels": rows[i]["label"]} for i in range(len(rows))]
    coll = lambda b: collate(b, tok.pad_token_id, 16)  # noqa: E731
    tr = prepare_data_loader(torch.utils.data.DataLoader(encode(sp["train"]), batch_size=cfg["batch_size"],
                                                         shuffle=True, collate_fn=coll, drop_last=True))
    va = prepare_data_loader(torch.utils.data.DataLoader(encode(sp["validation"]), batch_size=64, collate_fn=coll))
    model = SentimentModel(cfg["model"], cfg["lr"], len(tr) * cfg["epochs"], tok.vocab_size)
    trainer = L.Trainer(max_epochs=cfg["epochs"], devices="auto", accelerator="auto", precision="bf16-mixed",
                        strategy=L.RayDDPStrategy(), plugins=[L.RayLightningEnvironment()],
                        callbacks=[L.RayTrainReportCallback()], enable_progress_bar=False,
                        limit_train_batches=cfg.get("max_steps"))
    trainer = L.prepare_trainer(trainer)
    trainer.fit(model, train_dataloaders=tr, val_dataloaders=va)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-workers", type=int, default=int(os.environ.get("MXTRAIN_RAY_NUM_WORKERS", "1")))
    ap.add_argument("--model", default="bert-base-cased")
    ap.add_argument("--epochs", type=int, default=int(os.environ.get("NUM_EPOCHS", "3")))
    ap.add_argument("--batch-size", type=int, default=16)
    ap.add_argument("--lr", type=float, default=1e-5)
    ap.add_argument("--train-size", type=int, default=3668)
    ap.add_argument("--eval-size", type=int, default=408)
    ap.add_argument("--max-steps", type=int, default=None)
    ap.add_argument("--storage-path", default=os.path.join(os.environ.get("HOME", "."), "ray_results"))
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args(argv)
    use_gpu = not a.cpu and torch.cuda.is_available() and os.environ.get("MXTRAIN_CPU_ONLY") != "1"
    cache = os.environ.get("MXTRAIN_CACHE", os.path.join(os.path.expanduser("~"), ".cache", "mxtrain"))
    trainer = TorchTrainer(train_func,
                           train_loop_config={"model": a.model, "epochs": a.epochs, "batch_size": a.batch_size,
                                              "lr": a.lr, "train_size": a.train_size, "eval_size": a.eval_size,
                                              "max_steps": a.max_steps, "cache": cache},
                           scaling_config=ScalingConfig(num_workers=a.num_workers, use_gpu=use_gpu),
                           run_config=RunConfig(name="ptl-sent-classification", storage_path=a.storage_path,
                                                checkpoint_config=CheckpointConfig(num_to_keep=1)))
    result = trainer.fit()
    print(f"Training result: {json.dumps(result.metrics)}", flush=True)
    print(f"Checkpoint: {result.checkpoint}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

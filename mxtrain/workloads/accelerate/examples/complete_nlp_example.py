"""BERT sequence classification on GLUE MRPC with Hugging Face Accelerate -- the workload
the reference's elastic example runs (`torchrun $DISTRIBUTED_ARGS
examples/complete_nlp_example.py --mixed_precision fp16 --checkpointing_steps epoch
--with_tracking --output_dir $CKPT_DIR --project_dir $PROJECT_DIR`,
examples/accelerate/bert-glue-mrpc/pretrain.yaml:42-51).

Same command line and behaviour (epochs of train + eval, `save_state` checkpoints every
N steps or every epoch, `--resume_from_checkpoint`, metrics tracking under
`--project_dir`), with mxtrain's MI355X BERT (HIP flash attention with key-padding
lengths, fused BDA-LayerNorm, bias-GeLU) instead of the CUDA model, and offline data
(mxtrain.data.glue: MRPC-shaped synthetic pairs, WordPiece vocabulary of
bert-base-cased's size, random-init weights).  ``--mixed_precision fp16|bf16`` runs
the bf16 kernel path on the GPU (no GradScaler needed).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))))))

import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

MAX_GPU_BATCH_SIZE = 16
EVAL_BATCH_SIZE = 32


def _f1_acc(preds, refs):
    preds, refs = preds.long(), refs.long()
    acc = (preds == refs).float().mean().item()
    tp = ((preds == 1) & (refs == 1)).sum().item()
    fp = ((preds == 1) & (refs == 0)).sum().item()
    fn = ((preds == 0) & (refs == 1)).sum().item()
    f1 = 2 * tp / max(2 * tp + fp + fn, 1)
    return {"accuracy": acc, "f1": f1}


class JsonlTracker:
    """Tracker used by --with_tracking when no TensorBoard/W&B is installed: one JSON line
    per `log` call under <project_dir>/<run>/metrics.jsonl."""

    def __init__(self, project_dir, run, is_main):
        self.path = os.path.join(project_dir, run, "metrics.jsonl") if is_main else None
        if self.path:
            os.makedirs(os.path.dirname(self.path), exist_ok=True)

    def store_init_configuration(self, cfg):
        if self.path:
            with open(os.path.join(os.path.dirname(self.path), "config.json"), "w") as f:
                json.dump(cfg, f, indent=1, default=str)

    def log(self, values, step=None):
        if self.path:
            with open(self.path, "a") as f:
                f.write(json.dumps(dict(values, step=step, time=time.time()), default=float) + "\n")


def get_dataloaders(accelerator, batch_size, tok_cache, sizes=None, seed=42):
    from mxtrain.data.glue import bert_tokenizer, collate, mrpc_splits
    splits = mrpc_splits(seed=0, sizes=sizes)
    with accelerator.main_process_first():
        tok = bert_tokenizer(tok_cache)

    def encode(rows):
        enc = tok([r["sentence1"] for r in rows], [r["sentence2"] for r in rows], truncation=True, max_length=512)
        return [{"input_ids": enc["input_ids"][i], "token_type_ids": enc["token_type_ids"][i],
                 "attention_mask": enc["attention_mask"][i], "labels": rows[i]["label"]} for i in range(len(rows))]

    train = encode(splits["train"])
    val = encode(splits["validation"])
    pad = tok.pad_token_id
    g = torch.Generator().manual_seed(seed)
    train_dl = DataLoader(train, shuffle=True, batch_size=batch_size, generator=g,
                          collate_fn=lambda b: collate(b, pad, 16), drop_last=False)
    eval_dl = DataLoader(val, shuffle=False, batch_size=EVAL_BATCH_SIZE, collate_fn=lambda b: collate(b, pad, 16))
    return train_dl, eval_dl, tok


def training_function(config, args):
    from accelerate import Accelerator
    from accelerate.utils import set_seed
    from mxtrain.models.bert import BERT_CONFIGS, BertConfig, BertForSequenceClassification

    mp = args.mixed_precision
    if mp in ("fp16", "bf16", "fp8"):
        # the model computes in bf16 itself on the GPU (HIP kernels are bf16): no autocast,
        # no loss scaling in Accelerate
        mp_acc = "no"
    else:
        mp_acc = mp
    accelerator = Accelerator(cpu=args.cpu, mixed_precision=mp_acc, project_dir=args.project_dir)
    if mp != mp_acc:
        accelerator.print(f"[mxtrain] --mixed_precision {mp}: bf16 compute inside the model (MI355X kernels)")
    if hasattr(args.checkpointing_steps, "isdigit"):
        if args.checkpointing_steps == "epoch":
            checkpointing_steps = "epoch"
        elif args.checkpointing_steps.isdigit():
            checkpointing_steps = int(args.checkpointing_steps)
        else:
            raise ValueError(f"--checkpointing_steps {args.checkpointing_steps}: expected 'epoch' or an int")
    else:
        checkpointing_steps = None
    lr, num_epochs, seed, batch_size = config["lr"], int(config["num_epochs"]), int(config["seed"]), int(config["batch_size"])
    tracker = None
    if args.with_tracking:
        run = os.path.split(__file__)[-1].split(".")[0]
        tracker = JsonlTracker(args.project_dir or ".", run, accelerator.is_main_process)
        tracker.store_init_configuration(config)
    gradient_accumulation_steps = 1
    if batch_size > MAX_GPU_BATCH_SIZE and accelerator.distributed_type != "XLA":
        gradient_accumulation_steps = batch_size // MAX_GPU_BATCH_SIZE
        batch_size = MAX_GPU_BATCH_SIZE
    set_seed(seed)
    tok_cache = os.path.join(os.environ.get("MXTRAIN_CACHE", os.path.join(os.path.expanduser("~"), ".cache", "mxtrain")),
                             f"{args.model}-wordpiece")
    sizes = {"train": args.train_size, "validation": args.eval_size} if args.train_size else None
    train_dl, eval_dl, tok = get_dataloaders(accelerator, batch_size, tok_cache, sizes, seed)
    mcfg = BertConfig(**BERT_CONFIGS[args.model])
    mcfg.vocab_size = max(mcfg.vocab_size, tok.vocab_size)
    model = BertForSequenceClassification(mcfg, seed=seed).to(accelerator.device)
    optimizer = torch.optim.AdamW(params=model.parameters(), lr=lr,
                                  fused=accelerator.device.type == "cuda")
    total_steps = (len(train_dl) * num_epochs) // gradient_accumulation_steps
    warmup = 100

    def lr_lambda(step):
        if step < warmup:
            return step / max(1, warmup)
        return max(0.0, (total_steps - step) / max(1, total_steps - warmup))

    lr_scheduler = torch.optim.lr_scheduler.LambdaLR(optimizer, lr_lambda)
    model, optimizer, train_dl, eval_dl, lr_scheduler = accelerator.prepare(
        model, optimizer, train_dl, eval_dl, lr_scheduler)

    overall_step = 0
    starting_epoch = 0
    resume_step = None
    if args.resume_from_checkpoint:
        path = args.resume_from_checkpoint
        if path == "latest" or not os.path.isdir(path):
            base = args.output_dir or "."
            cands = [os.path.join(base, d) for d in os.listdir(base)
                     if d.startswith(("epoch_", "step_")) and os.path.isdir(os.path.join(base, d))] \
                if os.path.isdir(base) else []
            path = max(cands, key=os.path.getctime) if cands else None
        if path:
            accelerator.print(f"Resumed from checkpoint: {path}")
            accelerator.load_state(path)
            name = os.path.basename(path.rstrip("/"))
            if name.startswith("epoch_"):
                starting_epoch = int(name[len("epoch_"):]) + 1
            else:
                resume_step = int(name[len("step_"):])
                starting_epoch = resume_step // len(train_dl)
                resume_step -= starting_epoch * len(train_dl)
            overall_step = starting_epoch * len(train_dl) + (resume_step or 0)

    for epoch in range(starting_epoch, num_epochs):
        model.train()
        total_loss = torch.zeros((), device=accelerator.device)
        t0 = time.time()
        nsamples = 0
        dl = train_dl
        if resume_step is not None and epoch == starting_epoch:
            dl = accelerator.skip_first_batches(train_dl, resume_step)
        for step, batch in enumerate(dl):
            out = model(**batch)
            loss = out["loss"] / gradient_accumulation_steps
            total_loss += loss.detach()
            accelerator.backward(loss)
            nsamples += batch["input_ids"].shape[0]
            if step % gradient_accumulation_steps == 0:
                optimizer.step()
                lr_scheduler.step()
                optimizer.zero_grad()
            overall_step += 1
            if isinstance(checkpointing_steps, int) and overall_step % checkpointing_steps == 0:
                accelerator.save_state(os.path.join(args.output_dir or ".", f"step_{overall_step}"))
            if args.max_train_steps and overall_step >= args.max_train_steps:
                break
        if accelerator.device.type == "cuda":
            torch.cuda.synchronize()
        train_time = time.time() - t0
        model.eval()
        preds, refs = [], []
        for batch in eval_dl:
            with torch.no_grad():
                logits = model(**{k: v for k, v in batch.items() if k != "labels"})["logits"]
            p, r = accelerator.gather_for_metrics((logits.argmax(-1), batch["labels"]))
            preds.append(p)
            refs.append(r)
        metric = _f1_acc(torch.cat(preds).cpu(), torch.cat(refs).cpu())
        sps = nsamples * accelerator.num_processes / max(train_time, 1e-9)
        accelerator.print(f"epoch {epoch}:", metric, f"train_loss {total_loss.item() / max(len(dl), 1):.4f}",
                          f"samples/s {sps:.1f}")
        if tracker is not None:
            tracker.log({"accuracy": metric["accuracy"], "f1": metric["f1"],
                         "train_loss": total_loss.item() / max(len(dl), 1), "epoch": epoch,
                         "samples_per_s": sps}, step=epoch)
        if checkpointing_steps == "epoch":
            accelerator.save_state(os.path.join(args.output_dir or ".", f"epoch_{epoch}"))
        if args.max_train_steps and overall_step >= args.max_train_steps:
            break
    accelerator.wait_for_everyone()
    accelerator.end_training()
    return metric


def main(argv=None):
    p = argparse.ArgumentParser(description="Simple example of training script.")
    p.add_argument("--mixed_precision", type=str, default=None, choices=["no", "fp16", "bf16", "fp8"])
    p.add_argument("--cpu", action="store_true", help="If passed, will train on the CPU.")
    p.add_argument("--checkpointing_steps", type=str, default=None)
    p.add_argument("--resume_from_checkpoint", type=str, default=None)
    p.add_argument("--with_tracking", action="store_true")
    p.add_argument("--output_dir", type=str, default=".")
    p.add_argument("--project_dir", type=str, default="logs")
    # mxtrain additions (defaults = the upstream example's hard-coded config)
    p.add_argument("--model", default="bert-base-cased")
    p.add_argument("--num_epochs", type=int, default=3)
    p.add_argument("--batch_size", type=int, default=16)
    p.add_argument("--lr", type=float, default=2e-5)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--max_train_steps", type=int, default=None)
    p.add_argument("--train_size", type=int, default=None)
    p.add_argument("--eval_size", type=int, default=64)
    args = p.parse_args(argv)
    args.mixed_precision = args.mixed_precision or "no"
    if os.environ.get("MXTRAIN_CPU_ONLY") == "1" and not torch.cuda.is_available():
        args.cpu = True
    config = {"lr": args.lr, "num_epochs": args.num_epochs, "seed": args.seed, "batch_size": args.batch_size}
    training_function(config, args)


if __name__ == "__main__":
    main()

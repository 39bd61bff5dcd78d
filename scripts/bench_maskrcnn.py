"""Mask R-CNN R50-FPN training throughput (BASELINE config 3 metric: images/s) on the
local GPUs: synthetic COCO-shaped data (800 x <=1333 after resize), random-init weights,
the real training step (RPN + proposals + RoI heads + mask head + SGD).

    python scripts/bench_maskrcnn.py [--steps 40] [--warmup 10] [--batch 1] [--images 64]
Single process = 1 GPU; multi-GPU through torchrun / mpirun (one rank per GPU).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--images", type=int, default=64)
    ap.add_argument("--data", default="/tmp/mx_coco_bench")
    ap.add_argument("--workers", type=int, default=6)
    ap.add_argument("--out", default=None)
    ap.add_argument("--graph", choices=("auto", "0", "1"), default="auto",
                    help="whole-step hipGraph replay (train.py --mx-graph; auto = on for 1 GPU)")
    ap.add_argument("--set", action="append", default=[],
                    help="A/B hook: module:attr=int (e.g. mxtrain.models.maskrcnn:MaskRCNN.fused_targets=0) or "
                         "lib:setter=int (a kernel-library setter, e.g. lib:mx_flash_dropmask_variant=0)")
    ap.add_argument("extra", nargs="*")
    a = ap.parse_args()
    rank = int(os.environ.get("RANK", os.environ.get("OMPI_COMM_WORLD_RANK", "0")))
    if rank == 0 and not os.path.exists(os.path.join(a.data, "annotations", "instances_train2017.json")):
        from mxtrain.data.coco_synth import write_split
        write_split(a.data, "train2017", a.images, 0, 1)
        write_split(a.data, "val2017", 4, 1, 1_000_000)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist  # data written by rank 0 before the others read it
        import time
        while not os.path.exists(os.path.join(a.data, "annotations", "instances_val2017.json")):
            time.sleep(0.5)
    for kv in a.set:
        import importlib
        target, val = kv.split("=")
        mod, attr = target.split(":")
        if mod == "lib":
            from mxtrain.ops import _lib
            _lib._fn(attr)(int(val))
        else:
            obj = importlib.import_module(mod)
            *path, last = attr.split(".")          # module:Class.attr reaches class attributes
            for n in path:
                obj = getattr(obj, n)
            setattr(obj, last, type(getattr(obj, last))(int(val)))
    from mxtrain.workloads.maskrcnn import train
    out = a.out or os.path.join(REPO, "gpurun_out", "maskrcnn_bench.jsonl")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    args = ["--logdir", "/tmp/mx_mrcnn_log", "--mx-max-steps", str(a.steps), "--mx-warmup-steps", str(a.warmup),
            "--throughput_log_freq", "10", "--mx-bench-json", out, "--mx-graph", a.graph, "--config", "MODE_MASK=True", "MODE_FPN=True",
            f"DATA.BASEDIR={a.data}", "TRAINER=horovod", f"TRAIN.BATCH_SIZE_PER_GPU={a.batch}",
            f"TRAIN.STEPS_PER_EPOCH={a.steps}", "TRAIN.EVAL_PERIOD=1000", "TRAIN.CHECKPOINT_PERIOD=1000",
            f"DATA.NUM_WORKERS={a.workers}", "DATA.VAL=()"] + a.extra
    import shutil
    shutil.rmtree("/tmp/mx_mrcnn_log", ignore_errors=True)
    return train.main(args)


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Interleaved same-box A/B of Mask R-CNN training throughput: ROUNDS x (A, B) child runs of
scripts/bench_maskrcnn.py, A with the --set hooks of --a, B with those of --b (each a
comma-separated list of module:attr=int / lib:setter=int), median img/s per arm.
    python scripts/mrcnn_ab.py --a "" --b "mxtrain.models.maskrcnn:MaskRCNN.fused_targets=0" --batch 4 --rounds 3"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default="")
    ap.add_argument("--b", default="")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    a = ap.parse_args()
    res = {"A": [], "B": []}
    for r in range(a.rounds):
        for tag, sets in (("A", a.a), ("B", a.b)):
            out = tempfile.mktemp(suffix=".jsonl")
            cmd = [sys.executable, os.path.join(REPO, "scripts", "bench_maskrcnn.py"), "--batch", str(a.batch),
                   "--steps", str(a.steps), "--warmup", str(a.warmup), "--out", out]
            for kv in filter(None, sets.split(",")):
                cmd += ["--set", kv]
            subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
            with open(out) as f:
                v = json.loads(f.read().strip().splitlines()[-1])["value"]
            os.remove(out)
            res[tag].append(v)
            print(f"round {r} {tag}: {v:.2f} img/s", flush=True)
    ma, mb = statistics.median(res["A"]), statistics.median(res["B"])
    print(f"A [{a.a}] {ma:.2f} img/s  B [{a.b}] {mb:.2f} img/s  B/A {mb / ma:.4f}  ({a.batch} img/GPU)")


if __name__ == "__main__":
    main()

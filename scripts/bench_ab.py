#!/usr/bin/env python3
"""Interleaved same-box A/B of the GPT-2 bench step: ROUNDS x (A, B) child runs of
`bench.py --no-maskrcnn --no-extra-configs` with the extra flags of --a / --b, median
tokens/s and ms/step per arm.
    python scripts/bench_ab.py --b "--no-wgrad-stream" --rounds 3 --steps 20
(a "+" in --a / --b separates arguments too: --b=--model=gpt3-6.7b+--no-defer-update)"""
import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", default="")
    ap.add_argument("--b", default="")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    res = {"A": [], "B": []}
    for r in range(a.rounds):
        for tag, extra in (("A", a.a), ("B", a.b)):
            cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", str(a.steps),
                   "--warmup", str(a.warmup), "--no-maskrcnn", "--no-extra-configs"] + shlex.split(extra.replace("+", " "))
            out = subprocess.run(cmd, check=True, stdout=subprocess.PIPE, text=True).stdout
            rec = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
            res[tag].append((rec["value"], rec["ms_per_step"]))
            print(f"round {r} {tag}: {rec['value']:.0f} tok/s {rec['ms_per_step']:.3f} ms/step", flush=True)
    for tag, extra in (("A", a.a), ("B", a.b)):
        v = statistics.median(x[0] for x in res[tag])
        ms = statistics.median(x[1] for x in res[tag])
        print(f"{tag} [{extra}] {v:.0f} tok/s {ms:.3f} ms/step")
    va = statistics.median(x[0] for x in res["A"])
    vb = statistics.median(x[0] for x in res["B"])
    print(f"B/A {vb / va:.4f}")


if __name__ == "__main__":
    main()

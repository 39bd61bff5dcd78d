"""Minimum end-to-end slice on an MI355X: the shipped example values files
through the launcher -- data-process(wikicorpus) then pytorchjob-distributed
(pretrain-ddp-zero1) with the full GPT-2 345M model on N local GPUs; only the iteration
count / intervals are cut so it finishes in minutes.  Logs are copied to gpurun_out/slice.

    python scripts/gpu_slice.py [--gpus 1] [--iters 60] [--docs 4000] [--example pretrain-ddp-zero1]
"""
import argparse
import os
import shutil
import sys
import time

import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
EX = os.path.join(REPO, "examples", "megatron-deepspeed", "gpt2_345m")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--docs", type=int, default=4000)
    ap.add_argument("--example", default="pretrain-ddp-zero1")
    ap.add_argument("--home", default="/tmp/mxhome")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "slice"))
    a = ap.parse_args()
    os.environ["MXTRAIN_HOME"] = a.home
    os.environ["NUM_DOCS"] = str(a.docs)
    os.makedirs(a.out, exist_ok=True)
    from mxtrain.launch import release as rel

    tmp = os.path.join(a.home, "values")
    os.makedirs(tmp, exist_ok=True)
    # data
    wk = yaml.safe_load(open(os.path.join(EX, "wikicorpus.yaml")))
    p = os.path.join(tmp, "wikicorpus.yaml")
    yaml.safe_dump(wk, open(p, "w"))
    t0 = time.time()
    st = rel.install(os.path.join(REPO, "charts/machine-learning/data-prep/data-process"), "mds-gpt2-345m",
                     value_files=[p], wait=True, timeout=900)
    open(os.path.join(a.out, "data-process.log"), "w").write(rel.logs("mds-gpt2-345m"))
    print(f"data-process: {st['phase']} in {time.time() - t0:.0f}s", flush=True)
    if st["phase"] != "Succeeded":
        return 1
    rel.uninstall("mds-gpt2-345m")
    # train
    doc = yaml.safe_load(open(os.path.join(EX, f"{a.example}.yaml")))
    pre = []
    for line in doc["pre_script"]:
        line = line.replace("--train-iters 500000", f"--train-iters {a.iters}")
        line = line.replace("--lr-decay-iters 320000", f"--lr-decay-iters {a.iters}")
        if line.startswith("export OUTPUT_ARGS="):
            line = (f'export OUTPUT_ARGS="--log-interval 10 --save-interval {a.iters} --eval-interval {a.iters // 2} '
                    f'--eval-iters 2 --mx-graph"')
        pre.append(line)
    doc["pre_script"] = pre
    doc["resources"]["nproc_per_node"] = a.gpus
    doc["resources"]["requests"] = {"amd.com/gpu": a.gpus}
    doc["resources"]["limits"] = {"amd.com/gpu": a.gpus}
    p = os.path.join(tmp, f"{a.example}.yaml")
    yaml.safe_dump(doc, open(p, "w"))
    t0 = time.time()
    st = rel.install(os.path.join(REPO, "charts/machine-learning/training/pytorchjob-distributed"), "mds-gpt2-345m",
                     value_files=[p], wait=True, timeout=1800)
    log = rel.logs("mds-gpt2-345m")
    open(os.path.join(a.out, f"{a.example}.log"), "w").write(log)
    print(f"{a.example}: {st['phase']} in {time.time() - t0:.0f}s", flush=True)
    print("\n".join(line for line in log.splitlines() if "iteration" in line or "loss" in line or "GPT" in line)[-4000:])
    ck = os.path.join(a.home, "pv", "pv-fsx", "home", "mds-gpt2-345m", "checkpoints", "0")
    if os.path.isdir(ck):
        with open(os.path.join(a.out, "checkpoint_tree.txt"), "w") as f:
            for root, dirs, files in os.walk(ck):
                for fn in sorted(files):
                    q = os.path.join(root, fn)
                    f.write(f"{os.path.relpath(q, ck)}\t{os.path.getsize(q)}\n")
    mdir = os.path.join(a.home, "pv", "pv-efs", "home", "mds-gpt2-345m", "logs", "0")
    if os.path.isdir(mdir):
        for fn in os.listdir(mdir):
            if fn.endswith((".jsonl", ".log")):
                shutil.copy(os.path.join(mdir, fn), a.out)
    return 0 if st["phase"] == "Succeeded" else 1


if __name__ == "__main__":
    sys.exit(main())

"""Node acceptance checks -- the single-node counterpart of the reference's cluster smoke
tests (eks-cluster/tests/test-gpu.yaml: GPUs visible + FSx mounted; test-gpu-efa.yaml:
a pod pair for manual NCCL tests).

    python -m mxtrain.runtime.nodecheck [--gpus N] [--json out.json] [--skip-collectives]

Checks, each reported with a measured number:
  * GPU inventory from the KFD topology (gfx target, HBM size) -- no HIP init in the parent;
  * per-GPU HBM stream bandwidth and bf16 GEMM throughput (one child process per GPU);
  * RCCL all-reduce / all-gather / reduce-scatter bus bandwidth across the N local GPUs
    (one rank per GPU, torch.distributed "nccl" = RCCL over xGMI) -- the nccl-tests run
    the reference leaves to the user;
  * the PV root (local NVMe standing in for /fsx, /efs) is writable, with its free space.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time


def kfd_inventory():
    gpus = []
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"), key=lambda x: int(x.split("/")[-2])):
        try:
            props = dict(l.split() for l in open(p) if len(l.split()) == 2)
        except OSError:
            continue
        gfx = int(props.get("gfx_target_version", "0"))
        if gfx == 0:
            continue
        node = os.path.dirname(p)
        mem = 0
        for mp in glob.glob(os.path.join(node, "mem_banks", "*", "properties")):
            try:
                mprops = dict(l.split() for l in open(mp) if len(l.split()) == 2)
                mem = max(mem, int(mprops.get("size_in_bytes", "0")))
            except OSError:
                pass
        gpus.append({"gfx_target_version": gfx, "simd_count": int(props.get("simd_count", "0")),
                     "hbm_gib": round(mem / 2 ** 30, 1)})
    return gpus


_DEVICE_PROBE = r"""
import json, sys, time, torch
dev = torch.device("cuda", 0)
n = 1 << 28
a = torch.empty(n, dtype=torch.float32, device=dev); b = torch.empty_like(a)
for _ in range(3): b.copy_(a)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(20): b.copy_(a)
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
bw = 2 * n * 4 / dt / 1e12
M = 8192
x = torch.randn(M, M, dtype=torch.bfloat16, device=dev); y = torch.randn(M, M, dtype=torch.bfloat16, device=dev)
for _ in range(3): x @ y
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(20): x @ y
torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
print(json.dumps({"name": torch.cuda.get_device_name(0), "hbm_copy_tb_s": round(bw, 2),
                  "bf16_gemm_8k_tflops": round(2 * M ** 3 / dt / 1e12, 1),
                  "hbm_total_gib": round(torch.cuda.get_device_properties(0).total_memory / 2 ** 30, 1)}))
"""

_COLL_PROBE = r"""
import json, os, time, torch, torch.distributed as dist
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
# one GPU per process: spawned with HIP_VISIBLE_DEVICES=<rank> (local) or under torchrun
lr = int(os.environ.get("LOCAL_RANK", "0")) if torch.cuda.device_count() > 1 else 0
torch.cuda.set_device(lr)
dev = torch.device("cuda", lr)
dist.init_process_group("nccl", rank=r, world_size=w, device_id=dev)
out = {}
for mb in (16, 256):
    n = mb * 2 ** 20 // 2
    t = torch.ones(n, dtype=torch.bfloat16, device=dev)
    g = torch.empty(n * w, dtype=torch.bfloat16, device=dev)
    s = torch.empty(n // w, dtype=torch.bfloat16, device=dev)
    for name, fn, factor in (("all_reduce", lambda: dist.all_reduce(t), 2 * (w - 1) / w),
                             ("all_gather", lambda: dist.all_gather_into_tensor(g, t), (w - 1) / w * w),
                             ("reduce_scatter", lambda: dist.reduce_scatter_tensor(s, t), (w - 1) / w)):
        for _ in range(3): fn()
        torch.cuda.synchronize(); dist.barrier()
        t0 = time.perf_counter()
        for _ in range(10): fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        out[f"{name}_{mb}MB_busbw_gb_s"] = round(n * 2 * factor / dt / 1e9, 1)
if os.environ.get("MXTRAIN_XGMI", "0") in ("1", "auto") and w <= 8:
    # the direct peer-to-peer kernels, checked against RCCL and timed per size
    from mxtrain.parallel.xgmi import XGMICommunicator, XGMIUnavailable
    try:
        c = XGMICommunicator(dist.group.WORLD, dev, max_bytes=256 << 20)
        res = c.autotune(sizes=(1 << 20, 16 << 20, 64 << 20))
        out["xgmi_ok"] = c.autotune_ok
        out["xgmi_vs_rccl_ms"] = {f"{op}_{nb >> 20}MB": [round(a, 4), round(b, 4)] for (op, nb), (a, b) in res.items()}
        c.close()
    except XGMIUnavailable as e:
        out["xgmi_ok"] = False
        out["xgmi_error"] = str(e)[:300]
if r == 0:
    print(json.dumps(out))
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def device_probe(gpu: int, timeout: int = 300):
    env = dict(os.environ, HIP_VISIBLE_DEVICES=str(gpu))
    r = subprocess.run([sys.executable, "-c", _DEVICE_PROBE], env=env, capture_output=True, text=True,
                       timeout=timeout)
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def collective_probe(n: int, timeout: int = 300):
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HIP_VISIBLE_DEVICES=str(r), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, "-c", _COLL_PROBE], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=timeout) for p in procs]
    if any(p.returncode for p in procs):
        return {"error": " | ".join(e[-300:] for _, e in outs if e)}
    return json.loads(outs[0][0].strip().splitlines()[-1])


def storage_probe():
    from .storage import pv_root
    root = pv_root()
    try:
        os.makedirs(root, exist_ok=True)
        with tempfile.NamedTemporaryFile(dir=root) as f:
            f.write(b"x" * (1 << 20))
            f.flush()
        du = shutil.disk_usage(root)
        return {"pv_root": root, "writable": True, "free_gib": round(du.free / 2 ** 30, 1)}
    except OSError as e:
        return {"pv_root": root, "writable": False, "error": str(e)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--skip-collectives", action="store_true")
    ap.add_argument("--skip-devices", action="store_true")
    ap.add_argument("--collectives-only", action="store_true",
                    help="this process is one rank of an external launch (torchrun / mpirun): run "
                         "only the collective probe in-process")
    a = ap.parse_args(argv)
    if a.collectives_only:
        exec(compile(_COLL_PROBE, "nodecheck-collectives", "exec"), {"__name__": "__nodecheck__"})
        return 0
    inv = kfd_inventory()
    n = a.gpus if a.gpus is not None else len(inv)
    rep = {"time": time.strftime("%Y-%m-%dT%H:%M:%S"), "gpus_found": len(inv), "inventory": inv,
           "storage": storage_probe()}
    if n and not a.skip_devices:
        rep["devices"] = [dict(gpu=i, **device_probe(i)) for i in range(n)]
    if n > 1 and not a.skip_collectives:
        rep["rccl"] = collective_probe(n)
    ok = rep["storage"].get("writable") and all("error" not in d for d in rep.get("devices", [])) and \
        "error" not in rep.get("rccl", {})
    rep["status"] = "PASS" if ok else "FAIL"
    print(json.dumps(rep, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

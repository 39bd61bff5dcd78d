"""Structured per-rank metrics stream + Megatron-style log lines.

``MetricsWriter`` appends one JSON object per record to
``<dir>/metrics-rank<R>.jsonl`` (step, loss, lr, grad-norm, tokens/s, samples/s,
TFLOP/s per GPU, HBM high-water mark, ...); ``megatron_line`` formats the familiar
``iteration N/ M | consumed samples: ... | lm loss: ...`` line the reference's logs
(`tee $OUTPUT_LOG`) are read for.  ``gpu_sample`` reads power / clocks / temperature
from the amdgpu sysfs hwmon nodes (no SMI process per sample); ``GPUSampler`` polls it on a
background thread for the rank's own GPU (found by PCI address) and reports mean / max
per logging interval, next to the DP communication time the optimizer measures
(``DistributedOptimizer.take_comm_ms``).
"""
from __future__ import annotations

import glob
import json
import os
import threading
import time
from typing import Dict, List, Optional

import torch


class MetricsWriter:
    def __init__(self, path_or_dir: Optional[str], rank: int = 0):
        self.path = None
        if path_or_dir:
            if path_or_dir.endswith(".jsonl"):
                self.path = path_or_dir
            else:
                os.makedirs(path_or_dir, exist_ok=True)
                self.path = os.path.join(path_or_dir, f"metrics-rank{rank}.jsonl")
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
        self.rank = rank

    def write(self, **rec):
        if not self.path:
            return
        rec.setdefault("time", time.time())
        rec.setdefault("rank", self.rank)
        with open(self.path, "a") as f:
            f.write(json.dumps(rec, default=float) + "\n")


def hbm_stats(device) -> dict:
    if device is None or getattr(device, "type", "cpu") != "cuda":
        return {}
    return {"hbm_max_allocated_gb": torch.cuda.max_memory_allocated(device) / 2 ** 30,
            "hbm_reserved_gb": torch.cuda.memory_reserved(device) / 2 ** 30}


def gpu_sample(card: int = 0, root: str = "/sys") -> dict:
    """Power (W), sclk/mclk (MHz), edge/junction temperature (C) from sysfs."""
    out = {}
    for hw in glob.glob(f"{root}/class/drm/card{card}/device/hwmon/hwmon*"):
        def rd(name, scale=1.0):
            p = os.path.join(hw, name)
            try:
                return float(open(p).read().strip()) * scale
            except (OSError, ValueError):
                return None
        for k, n, s in (("power_w", "power1_average", 1e-6), ("power_w", "power1_input", 1e-6),
                        ("temp_edge_c", "temp1_input", 1e-3), ("temp_junction_c", "temp2_input", 1e-3),
                        ("sclk_mhz", "freq1_input", 1e-6), ("mclk_mhz", "freq2_input", 1e-6)):
            v = rd(n, s)
            if v is not None and k not in out:
                out[k] = v
    return out


def megatron_line(iteration: int, train_iters: int, consumed: int, elapsed_ms: float, lr: float,
                  global_batch: int, loss: float, grad_norm: Optional[float], skipped: int = 0,
                  nan: int = 0, samples_per_sec: Optional[float] = None, tflops: Optional[float] = None,
                  tokens_per_sec: Optional[float] = None, loss_scale: float = 1.0) -> str:
    s = (f" iteration {iteration:8d}/{train_iters:8d} | consumed samples: {consumed:12d} |"
         f" elapsed time per iteration (ms): {elapsed_ms:.1f} | learning rate: {lr:.3E} |"
         f" global batch size: {global_batch:5d} | lm loss: {loss:.6E} | loss scale: {loss_scale:.1f} |")
    if grad_norm is not None:
        s += f" grad norm: {grad_norm:.3f} |"
    s += f" number of skipped iterations: {skipped:3d} | number of nan iterations: {nan:3d} |"
    if samples_per_sec is not None:
        s += f" samples per second: {samples_per_sec:.3f} |"
    if tokens_per_sec is not None:
        s += f" tokens per second: {tokens_per_sec:.1f} |"
    if tflops is not None:
        s += f" TFLOPs: {tflops:.2f} |"
    return s


def drm_card_for_device(device) -> Optional[int]:
    """The /sys/class/drm/card<N> of a torch GPU, matched by PCI address (robust to
    HIP_VISIBLE_DEVICES renumbering); None if unknown."""
    try:
        p = torch.cuda.get_device_properties(device)
        want = (getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
    except Exception:   # noqa: BLE001 -- CPU / no properties
        return None
    for d in glob.glob("/sys/class/drm/card[0-9]*"):
        if "-" in os.path.basename(d):
            continue
        try:
            addr = os.path.basename(os.path.realpath(os.path.join(d, "device")))   # 0000:03:00.0
            dom, bus, devfn = addr.split(":")
            dev = devfn.split(".")[0]
            if (int(dom, 16), int(bus, 16), int(dev, 16)) == want:
                return int(os.path.basename(d)[4:])
        except (OSError, ValueError):
            continue
    return None


class GPUSampler:
    """Background sysfs sampler (power / sclk / mclk / temperatures) of one GPU.
    ``take()`` -> {gpu_power_w_mean, gpu_power_w_max, gpu_sclk_mhz_mean, gpu_mclk_mhz_mean,
    gpu_temp_junction_c_max, gpu_samples} over the samples since the last call."""

    def __init__(self, card: Optional[int], interval_s: float = 0.5, root: str = "/sys"):
        self.card, self.interval, self.root = card, interval_s, root
        self._buf: List[Dict[str, float]] = []
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._t = None
        if card is not None and gpu_sample(card, root):
            self._t = threading.Thread(target=self._run, name="mx-gpu-sampler", daemon=True)
            self._t.start()

    def _run(self):
        while not self._stop.wait(self.interval):
            smp = gpu_sample(self.card, self.root)
            if smp:
                with self._lock:
                    self._buf.append(smp)

    def take(self) -> Dict[str, float]:
        with self._lock:
            buf, self._buf = self._buf, []
        if not buf:
            return {}

        def col(k):
            return [b[k] for b in buf if b.get(k) is not None]
        out = {"gpu_samples": len(buf)}
        for k, agg in (("power_w", "mean"), ("power_w", "max"), ("sclk_mhz", "mean"), ("mclk_mhz", "mean"),
                       ("temp_junction_c", "max"), ("temp_edge_c", "max")):
            v = col(k)
            if v:
                out[f"gpu_{k}_{agg}"] = (sum(v) / len(v)) if agg == "mean" else max(v)
        return out

    def close(self):
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2)

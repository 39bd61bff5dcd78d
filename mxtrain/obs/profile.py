"""Step-window profiling and debug modes for every workload.

Profiling (``mxtrain install --profile`` sets these for every replica, or set them by hand):

    MXTRAIN_PROFILE=torch          torch.profiler with ROCm activities over a step window
    MXTRAIN_PROFILE_STEPS=5:8      [start, stop) steps of the window (default 5:8)
    MXTRAIN_PROFILE_DIR=<dir>      default $HOME/logs/<HOSTNAME>/profile

Each rank writes ``trace-rank<R>.json`` (Chrome trace: HIP kernels, RCCL collectives,
host ops) and ``kernels-rank<R>.txt`` (per-kernel self-time table sorted by device time,
the same view as ``rocprofv3 --kernel-trace --stats``).  Kernel-counter runs (MFMA
utilisation, LDS bank conflicts, HBM bytes) are taken with ``rocprofv3 --pmc ... --
python3 <workload>`` directly on the worker command: a profiler must never wrap the
train-script's ``bash`` (its preloaded library would initialise the GPU before the exec
of python).

Debug mode (``mxtrain install --debug-mode``, or ``MXTRAIN_DEBUG=1``): ``debug_env()`` is
added to every replica's environment -- serialised kernel launches and synchronous HIP
errors (``AMD_SERIALIZE_KERNEL=3``, ``HIP_LAUNCH_BLOCKING=1``), collective consistency
checks (``TORCH_DISTRIBUTED_DEBUG=DETAIL``, ``TORCH_NCCL_ASYNC_ERROR_HANDLING=1``), RCCL
logging (``NCCL_DEBUG=INFO``), and ``MXTRAIN_CHECK_FINITE=1``, which makes the trainers
check loss and gradient norm for inf/nan every step and raise at the first bad step.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch


def debug_env() -> Dict[str, str]:
    return {
        "AMD_SERIALIZE_KERNEL": "3",
        "HIP_LAUNCH_BLOCKING": "1",
        "TORCH_DISTRIBUTED_DEBUG": "DETAIL",
        "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1",
        "NCCL_DEBUG": "INFO",
        "MXTRAIN_CHECK_FINITE": "1",
    }


def profile_env(mode: str = "torch", steps: str = "5:8") -> Dict[str, str]:
    return {"MXTRAIN_PROFILE": mode, "MXTRAIN_PROFILE_STEPS": steps}


def check_finite_enabled() -> bool:
    return os.environ.get("MXTRAIN_CHECK_FINITE", "0") == "1"


def check_finite(step: int, **values) -> None:
    """Raise on the first non-finite value (debug mode; synchronises)."""
    for k, v in values.items():
        f = float(v.detach().float().item()) if torch.is_tensor(v) else float(v)
        if f != f or f in (float("inf"), float("-inf")):
            raise FloatingPointError(f"non-finite {k} = {f} at step {step}")


class StepProfiler:
    """Call ``step(it)`` once per training iteration (after the step ran)."""

    def __init__(self, rank: int = 0, out_dir: Optional[str] = None, mode: Optional[str] = None,
                 steps: Optional[str] = None):
        self.mode = mode if mode is not None else os.environ.get("MXTRAIN_PROFILE", "")
        s = steps or os.environ.get("MXTRAIN_PROFILE_STEPS", "5:8")
        a, _, b = s.partition(":")
        self.start, self.stop = int(a), int(b or int(a) + 3)
        home = os.environ.get("HOME", ".")
        host = os.environ.get("HOSTNAME", "local")
        self.dir = out_dir or os.environ.get("MXTRAIN_PROFILE_DIR") or os.path.join(home, "logs", host, "profile")
        self.rank = rank
        self._prof = None
        self.done = False

    @property
    def enabled(self) -> bool:
        return self.mode == "torch"

    def step(self, it: int) -> None:
        if not self.enabled or self.done:
            return
        if self._prof is None and it >= self.start:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self._prof.__enter__()
            return
        if self._prof is not None and it >= self.stop:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._prof.__exit__(None, None, None)
            os.makedirs(self.dir, exist_ok=True)
            self._prof.export_chrome_trace(os.path.join(self.dir, f"trace-rank{self.rank}.json"))
            sort = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
            with open(os.path.join(self.dir, f"kernels-rank{self.rank}.txt"), "w") as f:
                f.write(self._prof.key_averages().table(sort_by=sort, row_limit=60))
            self._prof = None
            self.done = True

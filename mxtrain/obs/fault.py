"""Fault injection + hang watchdog (SURVEY §5.3 "New framework").

Fault injection: ``MXTRAIN_FAULT="<rank>:<step>:<kind>[,...]"`` with kind one of
``exit`` (exit code 17), ``kill`` (SIGKILL self), ``hang`` (sleep forever), ``raise``
(Python exception).  ``rank`` may be ``*``.  A fault fires once per process lifetime,
and -- so that gang-restart tests terminate -- only while ``MXTRAIN_FAULT_ONCE_FILE``
(if set) does not exist yet; the file is created when it fires.

Watchdog: each rank touches ``<dir>/heartbeat-rank<R>`` every step; a daemon thread
aborts the process (exit 124) when no heartbeat happened for ``timeout`` seconds, so a
rank stuck in a collective does not hang the job forever (the controller then applies
restartPolicy / backoffLimit).
"""
from __future__ import annotations

import os
import signal
import threading
import time
from typing import List, Optional, Tuple


def _parse(spec: str) -> List[Tuple[str, int, str]]:
    out = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        r, s, k = part.split(":")
        out.append((r, int(s), k))
    return out


class FaultInjector:
    def __init__(self, rank: int, spec: Optional[str] = None):
        self.rank = rank
        self.faults = _parse(spec if spec is not None else os.environ.get("MXTRAIN_FAULT", ""))
        self.once = os.environ.get("MXTRAIN_FAULT_ONCE_FILE")
        self.fired = False

    def maybe_fire(self, step: int):
        if self.fired or not self.faults:
            return
        for r, s, kind in self.faults:
            if (r == "*" or int(r) == self.rank) and s == step:
                if self.once:
                    if os.path.exists(self.once):
                        return
                    open(self.once, "w").write(f"{self.rank}:{step}:{kind}\n")
                self.fired = True
                print(f"[mxtrain.fault] rank {self.rank} step {step}: injecting {kind}", flush=True)
                if kind == "exit":
                    os._exit(17)
                if kind == "kill":
                    os.kill(os.getpid(), signal.SIGKILL)
                if kind == "hang":
                    while True:
                        time.sleep(3600)
                if kind == "raise":
                    raise RuntimeError(f"injected fault at step {step}")
                raise ValueError(f"unknown fault kind {kind}")


class Watchdog:
    def __init__(self, directory: Optional[str], rank: int, timeout: float):
        self.path = os.path.join(directory, f"heartbeat-rank{rank}") if directory else None
        if self.path:
            os.makedirs(directory, exist_ok=True)
        self.timeout = timeout
        self.last = time.time()
        self.step = 0
        self._stop = threading.Event()
        if timeout and timeout > 0:
            threading.Thread(target=self._run, daemon=True).start()

    def beat(self, step: int):
        self.last = time.time()
        self.step = step
        if self.path:
            with open(self.path, "w") as f:
                f.write(f"{step} {self.last:.3f}\n")

    def _run(self):
        while not self._stop.wait(min(5.0, self.timeout / 4)):
            if time.time() - self.last > self.timeout:
                print(f"[mxtrain.watchdog] no progress for {self.timeout:.0f}s after step {self.step}; "
                      "aborting rank", flush=True)
                os._exit(124)

    def stop(self):
        self._stop.set()

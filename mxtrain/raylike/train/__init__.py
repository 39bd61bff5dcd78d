"""Ray Train-style worker-group executor on one MI355X node (replaces KubeRay + Ray Train
for the raytrain chart).

    from mxtrain.raylike import train
    from mxtrain.raylike.train import ScalingConfig, RunConfig, CheckpointConfig
    from mxtrain.raylike.train.torch import TorchTrainer, prepare_model, prepare_data_loader

    def loop(config):
        ctx = train.get_context()            # world rank / size / local rank
        model = prepare_model(Net())         # device placement + DDP over RCCL
        ...
        train.report({"loss": l}, checkpoint=train.Checkpoint.from_directory(d))

    result = TorchTrainer(loop, train_loop_config={...},
                          scaling_config=ScalingConfig(num_workers=8, use_gpu=True),
                          run_config=RunConfig(name="r50", storage_path="/efs/ray_results")).fit()

``fit()`` serialises the loop with cloudpickle, starts ``num_workers`` rank processes
(one per GPU of the RayJob's worker group: MXTRAIN_RAY_GPUS, HIP_VISIBLE_DEVICES), gives
them the torch.distributed env (RCCL backend on GPUs, gloo on CPU), streams rank 0's
``report`` calls into ``<storage>/<name>/progress.jsonl`` and persists reported
checkpoints as ``<storage>/<name>/checkpoint_<NNNNNN>/``.  The returned ``Result`` has
``metrics`` (last report), ``checkpoint`` and ``path``; a failing worker fails the fit
(``TrainingFailedError``) after the group is torn down.
"""
from __future__ import annotations

import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import torch

_WORKER_ENV = "MXTRAIN_RAYLIKE_WORKER"


class TrainingFailedError(RuntimeError):
    pass


@dataclass
class ScalingConfig:
    num_workers: int = 1
    use_gpu: bool = False
    resources_per_worker: Optional[Dict[str, float]] = None
    trainer_resources: Optional[Dict[str, float]] = None
    placement_strategy: str = "PACK"


@dataclass
class CheckpointConfig:
    num_to_keep: Optional[int] = None
    checkpoint_score_attribute: Optional[str] = None
    checkpoint_score_order: str = "max"


@dataclass
class FailureConfig:
    max_failures: int = 0


@dataclass
class RunConfig:
    name: Optional[str] = None
    storage_path: Optional[str] = None
    checkpoint_config: CheckpointConfig = field(default_factory=CheckpointConfig)
    failure_config: FailureConfig = field(default_factory=FailureConfig)
    verbose: int = 1


class Checkpoint:
    def __init__(self, path: str):
        self.path = path

    @classmethod
    def from_directory(cls, path: str) -> "Checkpoint":
        return cls(os.path.abspath(path))

    def to_directory(self, path: Optional[str] = None) -> str:
        if path is None:
            return self.path
        shutil.copytree(self.path, path, dirs_exist_ok=True)
        return path

    def as_directory(self):
        import contextlib
        return contextlib.nullcontext(self.path)

    def __repr__(self):
        return f"Checkpoint(path={self.path!r})"


@dataclass
class Result:
    metrics: Dict[str, Any]
    checkpoint: Optional[Checkpoint]
    path: str
    error: Optional[BaseException] = None
    metrics_dataframe: Any = None
    best_checkpoints: List = field(default_factory=list)


# ---------------------------------------------------------------------------- worker side
class TrainContext:
    def get_world_rank(self) -> int:
        return int(os.environ.get("RANK", "0"))

    def get_world_size(self) -> int:
        return int(os.environ.get("WORLD_SIZE", "1"))

    def get_local_rank(self) -> int:
        return int(os.environ.get("LOCAL_RANK", "0"))

    def get_local_world_size(self) -> int:
        return int(os.environ.get("LOCAL_WORLD_SIZE", "1"))

    def get_node_rank(self) -> int:
        return 0

    def get_trial_name(self) -> str:
        return os.environ.get("MXTRAIN_RAYLIKE_NAME", "")

    def get_experiment_name(self) -> str:
        return os.environ.get("MXTRAIN_RAYLIKE_NAME", "")

    def get_storage(self):
        return os.environ.get("MXTRAIN_RAYLIKE_RUN_DIR", "")


_CTX = TrainContext()
_REPORTS = {"n": 0}


def get_context() -> TrainContext:
    return _CTX


def get_checkpoint() -> Optional[Checkpoint]:
    p = os.environ.get("MXTRAIN_RAYLIKE_RESUME")
    return Checkpoint(p) if p else None


def report(metrics: Dict[str, Any], checkpoint: Optional[Checkpoint] = None):
    """Rank 0's metrics (and checkpoint) are recorded; every rank must call it (it is a
    synchronisation point, as in Ray Train)."""
    import torch.distributed as dist
    run_dir = os.environ.get("MXTRAIN_RAYLIKE_RUN_DIR")
    if dist.is_initialized():
        dist.barrier()
    _REPORTS["n"] += 1
    if _CTX.get_world_rank() != 0 or not run_dir:
        return
    rec = {k: (float(v) if isinstance(v, (int, float)) or torch.is_tensor(v) else v) for k, v in metrics.items()}
    rec["training_iteration"] = _REPORTS["n"]
    rec["timestamp"] = time.time()
    if checkpoint is not None:
        dst = os.path.join(run_dir, f"checkpoint_{_REPORTS['n'] - 1:06d}")
        if os.path.abspath(checkpoint.path) != dst:
            shutil.copytree(checkpoint.path, dst, dirs_exist_ok=True)
        rec["checkpoint_dir_name"] = os.path.basename(dst)
    with open(os.path.join(run_dir, "progress.jsonl"), "a") as f:
        f.write(json.dumps(rec, default=str) + "\n")


def _worker_main(payload: str):
    import cloudpickle
    with open(payload, "rb") as f:
        fn, config = cloudpickle.load(f)
    from .torch import setup_process_group, teardown_process_group
    setup_process_group()
    try:
        if config is None:
            fn()
        else:
            fn(config)
    finally:
        teardown_process_group()


# ---------------------------------------------------------------------------- driver side
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gpu_pool() -> List[str]:
    env = os.environ.get("MXTRAIN_RAY_GPUS") or os.environ.get("HIP_VISIBLE_DEVICES") or ""
    ids = [x for x in env.split(",") if x.strip() != ""]
    if ids:
        return ids
    try:
        n = torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        n = 0
    return [str(i) for i in range(n)]


class DataParallelTrainer:
    def __init__(self, train_loop_per_worker: Callable, *, train_loop_config: Optional[dict] = None,
                 scaling_config: Optional[ScalingConfig] = None, run_config: Optional[RunConfig] = None,
                 datasets: Optional[dict] = None, resume_from_checkpoint: Optional[Checkpoint] = None, **_):
        self.fn = train_loop_per_worker
        self.config = train_loop_config
        self.scaling = scaling_config or ScalingConfig()
        self.run = run_config or RunConfig()
        self.resume = resume_from_checkpoint

    def fit(self) -> Result:
        import cloudpickle
        name = self.run.name or f"TorchTrainer_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        storage = self.run.storage_path or os.path.join(os.path.expanduser("~"), "ray_results")
        run_dir = os.path.join(storage, name)
        os.makedirs(run_dir, exist_ok=True)
        n = int(self.scaling.num_workers)
        gpus = _gpu_pool() if self.scaling.use_gpu else []
        if self.scaling.use_gpu and gpus and n > len(gpus):
            raise TrainingFailedError(f"ScalingConfig(num_workers={n}, use_gpu=True) needs {n} GPUs, "
                                      f"the worker group has {len(gpus)} ({','.join(gpus)})")
        fd, payload = tempfile.mkstemp(prefix="raylike-", suffix=".pkl", dir=run_dir)
        with os.fdopen(fd, "wb") as f:
            cloudpickle.dump((self.fn, self.config), f)
        port = _free_port()
        procs = []
        print(f"[mxtrain.raylike] starting worker group: {n} workers, "
              f"{'GPUs ' + ','.join(gpus[:n]) if gpus else 'CPU'}; results in {run_dir}", flush=True)
        for r in range(n):
            env = dict(os.environ)
            env.update({_WORKER_ENV: "1", "RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_RANK": str(r),
                        "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                        "MXTRAIN_RAYLIKE_RUN_DIR": run_dir, "MXTRAIN_RAYLIKE_NAME": name,
                        "HSA_ENABLE_IPC_MODE_LEGACY": env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")})
            if gpus:
                env["HIP_VISIBLE_DEVICES"] = ",".join(gpus[:n])
                env.pop("MXTRAIN_CPU_ONLY", None)
            else:
                env["MXTRAIN_CPU_ONLY"] = "1"
            if self.resume is not None:
                env["MXTRAIN_RAYLIKE_RESUME"] = self.resume.path
            pp = env.get("PYTHONPATH", "")
            repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            env["PYTHONPATH"] = repo + (os.pathsep + pp if pp else "")
            # the payload may reference functions of the driver's __main__ script
            main_file = getattr(sys.modules.get("__main__"), "__file__", None)
            if main_file:
                env["PYTHONPATH"] = os.path.dirname(os.path.abspath(main_file)) + os.pathsep + env["PYTHONPATH"]
            procs.append(subprocess.Popen([sys.executable, "-m", "mxtrain.raylike.train", payload], env=env,
                                          start_new_session=True))
        err = None
        try:
            while True:
                codes = [p.poll() for p in procs]
                bad = [(i, c) for i, c in enumerate(codes) if c not in (None, 0)]
                if bad:
                    err = TrainingFailedError(f"worker rank {bad[0][0]} exited with code {bad[0][1]}")
                    break
                if all(c == 0 for c in codes):
                    break
                time.sleep(0.2)
        finally:
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)
            os.unlink(payload)
        metrics, ckpt = {}, None
        prog = os.path.join(run_dir, "progress.jsonl")
        if os.path.exists(prog):
            lines = [json.loads(x) for x in open(prog) if x.strip()]
            if lines:
                metrics = lines[-1]
            cks = [l["checkpoint_dir_name"] for l in lines if "checkpoint_dir_name" in l]
            keep = self.run.checkpoint_config.num_to_keep
            if keep:
                for old in cks[:-keep]:
                    shutil.rmtree(os.path.join(run_dir, old), ignore_errors=True)
            if cks:
                ckpt = Checkpoint(os.path.join(run_dir, cks[-1]))
        res = Result(metrics=metrics, checkpoint=ckpt, path=run_dir, error=err)
        if err is not None:
            raise err
        return res


"""Megatron-DeepSpeed checkpoint layout writer/reader.

Directory layout (unchanged from Megatron-DeepSpeed + DeepSpeed ZeRO-1, so
`/fsx/home/<rel>/checkpoints/<node_rank>/...` trees look the same on MI355X)::

    <save>/latest                                   text: "global_step<N>"
    <save>/latest_checkpointed_iteration.txt        text: "<N>"
    <save>/global_step<N>/mp_rank_<MM>_model_states.pt
    <save>/global_step<N>/zero_pp_rank_<D>_mp_rank_<MM>_optim_states.pt

* ``mp_rank_MM`` = model-parallel rank (pp_rank * tp + tp_rank), written by the DP rank 0
  replica of that model-parallel slice (DeepSpeed semantics: with per-node save dirs,
  later nodes hold only their ZeRO shards);
* ``zero_pp_rank_D`` = data-parallel rank D's optimizer partition (fp32 master,
  exp_avg, exp_avg_sq of its 1/DP shard).

``module`` uses Megatron state-dict keys (``language_model.embedding.word_embeddings.
weight``, ``language_model.encoder.layers.<i>.self_attention.query_key_value.weight`` with
Megatron's per-head [q, k, v] interleave, ...), layer indices local to the stage, as
Megatron does.  Files contain only tensors / plain Python containers, so they load with
``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

from .models.gpt import GPTConfig, stage_layer_range

DS_VERSION = "0.13.4+mxtrain"

_LAYER_MAP = {
    "ln1_w": "input_layernorm.weight", "ln1_b": "input_layernorm.bias",
    "qkv_w": "self_attention.query_key_value.weight", "qkv_b": "self_attention.query_key_value.bias",
    "proj_w": "self_attention.dense.weight", "proj_b": "self_attention.dense.bias",
    "ln2_w": "post_attention_layernorm.weight", "ln2_b": "post_attention_layernorm.bias",
    "fc1_w": "mlp.dense_h_to_4h.weight", "fc1_b": "mlp.dense_h_to_4h.bias",
    "fc2_w": "mlp.dense_4h_to_h.weight", "fc2_b": "mlp.dense_4h_to_h.bias",
    "router_w": "mlp.deepspeed_moe.gate.wg.weight",
}
# expert tensors, one file per (layer, global expert id) as DeepSpeed MoE writes them:
# layer_<L>_expert_<E>_mp_rank_<MM>_model_states.pt
_EXPERT_MAP = {"fc1_w": "dense_h_to_4h.weight", "fc1_b": "dense_h_to_4h.bias",
               "fc2_w": "dense_4h_to_h.weight", "fc2_b": "dense_4h_to_h.bias"}
_LAYER_RMAP = {v: k for k, v in _LAYER_MAP.items()}


# ---------------------------------------------------------------------- qkv layout
def qkv_to_megatron(t: torch.Tensor, hl: int, kvl: int, D: int) -> torch.Tensor:
    """ours [q(hl*D); k(kvl*D); v(kvl*D)] -> Megatron per-group [q.. k v] interleave."""
    rest = t.shape[1:]
    q = t[: hl * D].reshape(kvl, hl // kvl, D, *rest)
    k = t[hl * D:(hl + kvl) * D].reshape(kvl, 1, D, *rest)
    v = t[(hl + kvl) * D:].reshape(kvl, 1, D, *rest)
    return torch.cat([q, k, v], 1).reshape(t.shape)


def qkv_from_megatron(t: torch.Tensor, hl: int, kvl: int, D: int) -> torch.Tensor:
    rest = t.shape[1:]
    g = t.reshape(kvl, hl // kvl + 2, D, *rest)
    q = g[:, : hl // kvl].reshape(hl * D, *rest)
    k = g[:, hl // kvl].reshape(kvl * D, *rest)
    v = g[:, hl // kvl + 1].reshape(kvl * D, *rest)
    return torch.cat([q, k, v], 0)


# ---------------------------------------------------------------------- name mapping
def to_megatron_state(params: Dict[str, torch.Tensor], cfg: GPTConfig, tp: int, pp: int,
                      pp_rank: int, host: bool = True) -> Dict[str, torch.Tensor]:
    l0, _ = stage_layer_range(cfg, pp, pp_rank)
    hl, kvl, D = cfg.num_attention_heads // tp, cfg.num_kv_heads // tp, cfg.head_dim
    out = {}
    for name, t in params.items():
        t = t.detach().cpu().clone() if host else t.detach()
        if name == "wte":
            out["language_model.embedding.word_embeddings.weight"] = t
        elif name == "wpe":
            out["language_model.embedding.position_embeddings.weight"] = t
        elif name == "wte_head":
            out["word_embeddings_for_head.weight"] = t
        elif name == "lm_head":
            out["language_model.output_layer.weight"] = t
        elif name.startswith("final_ln"):
            out["language_model.encoder.final_layernorm." + ("weight" if name.endswith("_w") else "bias")] = t
        elif name.startswith("layers."):
            _, i, leaf = name.split(".", 2)
            if leaf in ("qkv_w", "qkv_b"):
                t = qkv_to_megatron(t, hl, kvl, D)
            out[f"language_model.encoder.layers.{int(i) - l0}.{_LAYER_MAP[leaf]}"] = t
        else:
            out[name] = t
    return out


def from_megatron_state(sd: Dict[str, torch.Tensor], cfg: GPTConfig, tp: int, pp: int,
                        pp_rank: int) -> Dict[str, torch.Tensor]:
    l0, _ = stage_layer_range(cfg, pp, pp_rank)
    hl, kvl, D = cfg.num_attention_heads // tp, cfg.num_kv_heads // tp, cfg.head_dim
    out = {}
    for k, t in sd.items():
        if k == "language_model.embedding.word_embeddings.weight":
            out["wte"] = t
        elif k == "language_model.embedding.position_embeddings.weight":
            out["wpe"] = t
        elif k == "word_embeddings_for_head.weight":
            out["wte_head"] = t
        elif k == "language_model.output_layer.weight":
            out["lm_head"] = t
        elif k.startswith("language_model.encoder.final_layernorm."):
            out["final_ln_w" if k.endswith("weight") else "final_ln_b"] = t
        elif k.startswith("language_model.encoder.layers."):
            rest = k[len("language_model.encoder.layers."):]
            i, leafm = rest.split(".", 1)
            leaf = _LAYER_RMAP[leafm]
            if leaf in ("qkv_w", "qkv_b"):
                t = qkv_from_megatron(t, hl, kvl, D)
            out[f"layers.{int(i) + l0}.{leaf}"] = t
        else:
            out[k] = t
    return out


# ---------------------------------------------------------------------- save / load
def _mp_rank(ps) -> int:
    return ps.pp_rank * ps.tp + ps.tp_rank


def _grad_rank(ps) -> int:
    """Index of this rank's ZeRO-1 shard in its gradient (dp x cp) group."""
    return ps.dp_rank * ps.cp + ps.cp_rank


def _optim_state(opt, sched, partitions):
    return {
        "zero_stage": 1, "loss_scaler": None, "dynamic_loss_scale": False, "overflow": False,
        "clip_grad": opt.clip, "partition_count": [partitions],
        "base_optimizer_state": {
            "state": {0: {"step": opt.step_count, "exp_avg": opt.exp_avg.detach(),
                          "exp_avg_sq": opt.exp_avg_sq.detach()}},
            "param_groups": [{"lr": sched(opt.step_count), "betas": list(opt.betas), "eps": opt.eps,
                              "weight_decay": opt.wd, "params": [0]}]},
        "single_partition_of_fp32_groups": [opt.master.detach()],
        "mx_shard_layout": [[int(b.start), int(b.end), int(so), int(n)] for (b, fs, so, n) in opt.slices],
    }


def _load_optim(opt, path):
    o = torch.load(path, map_location="cpu", weights_only=True)["optimizer_state_dict"]
    base = o["base_optimizer_state"]["state"][0]
    opt.load_shard_state({"master": o["single_partition_of_fp32_groups"][0],
                          "exp_avg": base["exp_avg"], "exp_avg_sq": base["exp_avg_sq"],
                          "step": base["step"]})


def _expert_files(trainer, d, mp):
    """[(path, {our name: tensor view})] for this EP rank's experts."""
    out = []
    El = trainer.cfg.num_experts // trainer.tcfg.moe_expert_parallel_size
    for name, t in trainer.eflat.params.items():
        _, i, _, leaf = name.split(".", 3)
        for j in range(El):
            e = trainer.ep_rank * El + j
            out.append((os.path.join(d, f"layer_{int(i)}_expert_{e}_mp_rank_{mp:02d}_model_states.pt"),
                        f"language_model.encoder.layers.{int(i)}.mlp.deepspeed_moe.experts."
                        f"deepspeed_experts.{e}.{_EXPERT_MAP[leaf]}", name, j))
    return out


def _atomic_save(obj, path):
    tmp = path + f".tmp{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _map_tensors(obj, fn):
    """obj with every tensor t replaced by fn(t) (dicts / lists / tuples walked)."""
    if isinstance(obj, torch.Tensor):
        return fn(obj)
    if isinstance(obj, dict):
        return {k: _map_tensors(v, fn) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_map_tensors(v, fn) for v in obj)
    return obj


def _collect(save_dir: str, trainer, iteration: int, consumed_samples: int, args, ds_config):
    """[(path, state)] of this rank's files for global_step<iteration>; tensors are still the
    live (device) tensors or fresh device temporaries -- the caller copies them to host."""
    ps = trainer.ps
    trainer.sync_params()
    d = os.path.join(save_dir, f"global_step{iteration}")
    mp = _mp_rank(ps)
    opt = trainer.opt
    sched = opt.schedule
    lr_state = {"max_lr": sched.lr, "min_lr": sched.min_lr, "warmup_steps": sched.warmup,
                "num_steps": opt.step_count, "decay_steps": sched.decay, "decay_style": sched.style}
    files = []
    if ps.dp_rank == 0 and ps.cp_rank == 0:
        module = to_megatron_state(trainer.flat.params, trainer.cfg, ps.tp, ps.pp, ps.pp_rank, host=False)
        state = {
            "module": module, "buffer_names": [], "optimizer": None, "lr_scheduler": lr_state,
            "sparse_tensor_module_names": [], "skipped_steps": 0, "global_steps": iteration,
            "global_samples": consumed_samples, "dp_world_size": ps.dp, "mp_world_size": ps.tp * ps.pp,
            "ds_config": ds_config or {}, "ds_version": DS_VERSION, "args": args or {},
            "iteration": iteration, "checkpoint_version": 3.0,
            "rng_state": [{"torch_rng_state": torch.get_rng_state(),
                           # cloned on the current stream: an async snapshot's side-stream
                           # copy would otherwise read the live seed after the next step's
                           # advance (the rest of the state is fenced before the optimizer)
                           "mx_dropout_seed": trainer.seed.t.detach().clone()}],
            "mx_config": trainer.cfg.__dict__.copy(),
        }
        files.append((os.path.join(d, f"mp_rank_{mp:02d}_model_states.pt"), state))
    optim = {"optimizer_state_dict": _optim_state(opt, sched, ps.grad_world),
             "ds_config": ds_config or {}, "ds_version": DS_VERSION}
    files.append((os.path.join(d, f"zero_pp_rank_{_grad_rank(ps)}_mp_rank_{mp:02d}_optim_states.pt"), optim))
    if trainer.eflat is not None:
        eo = trainer.eopt
        edp_rank = _grad_rank(ps) // trainer.tcfg.moe_expert_parallel_size
        if edp_rank == 0:   # one replica of each expert set writes the expert files
            ef: Dict[str, Dict[str, torch.Tensor]] = {}
            for path, key, name, j in _expert_files(trainer, d, mp):
                ef.setdefault(path, {})[key] = trainer.eflat.params[name][j].detach()
            files.extend(ef.items())
        files.append((os.path.join(d, f"expp_rank_{trainer.ep_rank}_zero_pp_rank_{edp_rank}"
                                      f"_mp_rank_{mp:02d}_optim_states.pt"),
                      {"optimizer_state_dict": _optim_state(eo, sched, eo.world), "ds_version": DS_VERSION}))
    return d, files


def _commit(save_dir: str, iteration: int, local_leader: Optional[bool]):
    """Point `latest` at global_step<iteration> once EVERY rank's files are on disk
    (collective: a barrier before the leader writes, one after)."""
    if dist.is_initialized():
        dist.barrier()
    if local_leader is None:
        local_leader = int(os.environ.get("LOCAL_RANK", "0")) == 0
    if local_leader:
        for name, text in (("latest", f"global_step{iteration}"), ("latest_checkpointed_iteration.txt", str(iteration))):
            tmp = os.path.join(save_dir, f".{name}.tmp{os.getpid()}")
            with open(tmp, "w") as f:
                f.write(text)
            os.replace(tmp, os.path.join(save_dir, name))
    if dist.is_initialized():
        dist.barrier()


def save_checkpoint(save_dir: str, trainer, iteration: int, consumed_samples: int = 0,
                    args: Optional[dict] = None, ds_config: Optional[dict] = None,
                    local_leader: Optional[bool] = None) -> str:
    """Synchronous save.  Every rank calls this (collective barrier at the end)."""
    d, files = _collect(save_dir, trainer, iteration, consumed_samples, args, ds_config)
    os.makedirs(d, exist_ok=True)
    for path, state in files:
        _atomic_save(_map_tensors(state, lambda t: t.detach().cpu().clone()), path)
    _commit(save_dir, iteration, local_leader)
    return d


class AsyncCheckpointer:
    """Checkpoint writes that overlap training (the reference's Megatron-
    DeepSpeed image pulls DeepSpeed async-IO for this, containers/megatron-deepspeed/
    Dockerfile:12,16, and saves every --save-interval, examples/megatron-deepspeed/
    gpt2_345m/pretrain-ddp-zero1.yaml:55,83).

    ``save()`` snapshots this rank's model / ZeRO-shard tensors into pinned host buffers
    with device-to-host copies on a side HIP stream (the copy engines, no CU time), then a
    background thread serialises them in the unchanged DeepSpeed layout.  The host returns
    immediately; the GPU only waits for the snapshot copies before the next optimizer
    update touches the parameters / fp32 master / moments (``fence()``, called by the
    trainer).  ``latest`` is advanced by ``wait()`` -- at the next save or at the end of
    training -- after a barrier, so it never names a checkpoint some rank has not
    finished.  Pinned buffers are allocated on the first save and reused (the ZeRO shard of
    GPT-3 6.7B at DP 8 is ~13 GB; re-pinning per save would cost more than the copy)."""

    def __init__(self, trainer):
        self.trainer = trainer
        self.device = trainer.device
        self._cuda = self.device.type == "cuda"
        self._stream = torch.cuda.Stream(device=self.device) if self._cuda else None
        self._host: Dict[int, torch.Tensor] = {}
        self._thread: Optional[threading.Thread] = None
        self._err: Optional[BaseException] = None
        self._commit_args = None
        self._event = None
        self.last_snapshot_s = 0.0
        self.last_write_s = 0.0

    # ---------------------------------------------------------------- snapshot
    def _host_copy(self, slot: int, t: torch.Tensor) -> torch.Tensor:
        t = t.detach()
        if not t.is_cuda:
            return t.clone()
        h = self._host.get(slot)
        if h is None or h.shape != t.shape or h.dtype != t.dtype:
            h = self._host[slot] = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        src = t if t.is_contiguous() else t.contiguous()
        src.record_stream(self._stream)
        h.copy_(src, non_blocking=True)
        return h

    def save(self, save_dir: str, iteration: int, consumed_samples: int = 0, args: Optional[dict] = None,
             ds_config: Optional[dict] = None, local_leader: Optional[bool] = None) -> str:
        self.wait()
        t0 = time.time()
        d, files = _collect(save_dir, self.trainer, iteration, consumed_samples, args, ds_config)
        os.makedirs(d, exist_ok=True)
        counter = [0]

        def copy(t):
            counter[0] += 1
            return self._host_copy(counter[0], t)

        if self._cuda:
            main = torch.cuda.current_stream(self.device)
            self._stream.wait_stream(main)
            with torch.cuda.stream(self._stream):
                host_files = [(p, _map_tensors(s, copy)) for p, s in files]
                self._event = torch.cuda.Event()
                self._event.record(self._stream)
        else:
            host_files = [(p, _map_tensors(s, copy)) for p, s in files]
            self._event = None
        self.last_snapshot_s = time.time() - t0
        self._commit_args = (save_dir, iteration, local_leader)
        self._err = None
        self._thread = threading.Thread(target=self._write, args=(host_files, self._event), daemon=True,
                                        name=f"mx-ckpt-{iteration}")
        self._thread.start()
        return d

    def _write(self, host_files, event):
        t0 = time.time()
        try:
            if event is not None:
                event.synchronize()
            for path, state in host_files:
                _atomic_save(state, path)
        except BaseException as e:  # surfaced by wait() on the training thread
            self._err = e
        self.last_write_s = time.time() - t0

    def fence(self):
        """Make the current stream wait for the snapshot copies (before anything writes the
        parameters or optimizer state again).  Host never blocks; no-op without a save."""
        if self._event is not None and self._cuda:
            torch.cuda.current_stream(self.device).wait_event(self._event)
            self._event = None

    @property
    def pending(self) -> bool:
        return self._thread is not None

    def wait(self):
        """Finish the in-flight write (if any) and advance `latest` to it (collective)."""
        if self._thread is None:
            return
        self._thread.join()
        self._thread = None
        err, self._err = self._err, None
        save_dir, iteration, leader = self._commit_args
        self._commit_args = None
        # every rank learns whether ANY rank's write failed before the collective commit:
        # a rank that raised alone would leave the others blocked in _commit's barrier
        ok = err is None
        if dist.is_initialized() and dist.get_world_size() > 1:
            dev = self.device if dist.get_backend() == "nccl" else torch.device("cpu")
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = bool(int(flag.item()))
        if err is not None:
            raise RuntimeError(f"async checkpoint write failed: {err!r}") from err
        if not ok:
            raise RuntimeError(f"async checkpoint write of global_step{iteration} failed on another rank")
        _commit(save_dir, iteration, leader)


def latest_iteration(load_dir: str) -> Optional[int]:
    p = os.path.join(load_dir, "latest_checkpointed_iteration.txt")
    if os.path.exists(p):
        return int(open(p).read().strip())
    p = os.path.join(load_dir, "latest")
    if os.path.exists(p):
        return int(open(p).read().strip().replace("global_step", ""))
    return None


def load_checkpoint(load_dir: str, trainer, load_optim: bool = True) -> Optional[dict]:
    """Restore params (+ optimizer shards) from the newest checkpoint in load_dir.
    Returns {"iteration", "consumed_samples"} or None if there is none."""
    it = latest_iteration(load_dir)
    if it is None:
        return None
    ps = trainer.ps
    d = os.path.join(load_dir, f"global_step{it}")
    mp = _mp_rank(ps)
    opt_path = os.path.join(d, f"zero_pp_rank_{_grad_rank(ps)}_mp_rank_{mp:02d}_optim_states.pt")
    model_path = os.path.join(d, f"mp_rank_{mp:02d}_model_states.pt")
    info = {"iteration": it, "consumed_samples": 0}
    if os.path.exists(model_path):
        st = torch.load(model_path, map_location="cpu", weights_only=True)
        sd = from_megatron_state(st["module"], trainer.cfg, ps.tp, ps.pp, ps.pp_rank)
        trainer.flat.load_state_dict(sd)
        info["consumed_samples"] = int(st.get("global_samples", 0))
        trainer.opt._refresh_master()
    if trainer.eflat is not None:
        cache: Dict[str, Dict[str, torch.Tensor]] = {}
        for path, key, name, j in _expert_files(trainer, d, mp):
            if os.path.exists(path):
                if path not in cache:
                    cache[path] = torch.load(path, map_location="cpu", weights_only=True)
                trainer.eflat.params[name][j].copy_(cache[path][key].to(trainer.eflat.dtype))
        if cache:
            trainer.eopt._refresh_master()
        edp_rank = _grad_rank(ps) // trainer.tcfg.moe_expert_parallel_size
        ep_path = os.path.join(d, f"expp_rank_{trainer.ep_rank}_zero_pp_rank_{edp_rank}"
                                  f"_mp_rank_{mp:02d}_optim_states.pt")
        if load_optim and os.path.exists(ep_path):
            _load_optim(trainer.eopt, ep_path)
    if load_optim and os.path.exists(opt_path):
        _load_optim(trainer.opt, opt_path)
    elif not os.path.exists(model_path):
        raise FileNotFoundError(f"no model or optimizer state for mp_rank {mp} / dp_rank {ps.dp_rank} in {d}")
    if "consumed_samples" not in info or info["consumed_samples"] == 0:
        info["consumed_samples"] = it * trainer.global_batch
    trainer.iteration = it
    # dropout stream continues where it stopped (one advance per optimizer step)
    hid_seed, attn_seed = trainer.seed_bases(trainer.tcfg, ps)
    trainer.seed.set_step(hid_seed, trainer.opt.step_count, attn_seed=attn_seed)
    return info

"""Whole-step hipGraph replay for Mask R-CNN training (forward, backward, gradient clip,
SGD-momentum update in ONE graph launch per step).

Why: the eager step issues ~2100 kernels per iteration; at batch 4 the host needs
~37 ms to enqueue them while the GPU needs less, so the GPU idles on Python (measured:
host enqueue 37.2 ms + loader wait 9.2 ms per 48 ms step).  The model is written with
static per-step shapes (models/maskrcnn.py: fixed-size proposals, fixed 512 RoIs/image,
rank-based sampling, no nonzero()/host sync), so once the inputs have static shapes the
whole step is capturable:

* images: one padded canvas per orientation (data/coco.py ``collate``);
* ground truth: ``fixed_gt`` pads boxes/labels to ``max_gt`` slots;
* masks: packed per-instance crops of variable total size are copied into the prefix
  of a fixed-capacity device buffer the graph reads through the crop table.

So there is one graph per (batch, canvas) shape -- two for COCO -- captured lazily the
first time a shape is seen (that step runs eagerly: it also warms MIOpen/BLAS, the
anchor caches and the momentum buffers, none of which may be created during capture).

Data parallel, the capture decision is collective.  A capturing rank issues a different
collective sequence than a replaying one (an eager step's bucket all-reduces, a capture
that records but does not run them, an agreement), so every step starts with a host-side
handshake on a gloo control group -- one all-reduce MAX of [needs a capture, mask bytes]
(~0.1 ms of host time, no GPU synchronisation): when ANY rank meets a new shape, every
rank runs the eager step (the capturing ranks also record their graph), and every rank
grows the mask buffer to the largest payload together (dropping and recapturing its
graphs).  Ranks whose orientation sequences differ therefore stay in collective lockstep;
AspectGroupedSampler additionally gives every rank the same orientation per step, so in
training the captures happen on the same steps anyway.
Graphs share one memory pool (they never run concurrently and keep no state between
replays except the parameters and optimizer buffers, which live outside the pool).
The learning rate is a device scalar filled before each replay.

The reference trains this model eagerly under TensorFlow/Horovod
(examples/maskrcnn/train-maskrcnn-tensorpack.yaml); this replaces its per-op runtime
dispatch, not its math: ``sgd_momentum_`` is torch.optim.SGD's update (dampening 0,
no Nesterov), so eager and graph steps are interchangeable and checkpoints are the same.
"""
from __future__ import annotations

import os
import sys
from typing import Dict, List, Optional

import torch

LOSS_NAMES = ("rpn_cls_loss", "rpn_box_loss", "fastrcnn_cls_loss", "fastrcnn_box_loss", "maskrcnn_loss",
              "total_loss")
INPUT_KEYS = ("images", "hw", "gt_boxes", "gt_labels", "gt_count", "gt_mask_table")


@torch.no_grad()
def sgd_momentum_(opt: torch.optim.SGD, lr) -> None:
    """torch.optim.SGD's step with a tensor (device) learning rate: d = g + wd p,
    buf = m buf + d (buf starts at 0, so the first step gives buf = d), p -= lr buf."""
    for g in opt.param_groups:
        ps = [p for p in g["params"] if p.grad is not None]
        if not ps:
            continue
        grads = [p.grad for p in ps]
        if g["weight_decay"]:
            torch._foreach_add_(grads, ps, alpha=g["weight_decay"])
        bufs = []
        for p in ps:
            st = opt.state[p]
            if st.get("momentum_buffer") is None:
                assert not (p.is_cuda and torch.cuda.is_current_stream_capturing()), \
                    "momentum buffers must exist before capture"
                st["momentum_buffer"] = torch.zeros_like(p)
            bufs.append(st["momentum_buffer"])
        if g["momentum"]:
            torch._foreach_mul_(bufs, g["momentum"])
            torch._foreach_add_(bufs, grads)
            upd = bufs
        else:
            upd = grads
        if torch.is_tensor(lr):
            torch._foreach_add_(ps, torch._foreach_mul(upd, -lr))
        else:
            torch._foreach_add_(ps, upd, alpha=-lr)


class GraphedTrainStep:
    def __init__(self, model, opt: torch.optim.SGD, params: List[torch.Tensor], clip: float, device,
                 flat_capacity: int = 16 << 20, flat_master=None):
        self.model, self.opt, self.params, self.clip, self.device = model, opt, params, clip, device
        self.graphs: Dict[tuple, tuple] = {}
        # with a FlatMaster (models/compute_weights.py) the update is its fused clip + SGD
        # launch and the learning rate its device scalar
        self.fm = flat_master
        self.lr = flat_master.lr if flat_master is not None else torch.zeros((), dtype=torch.float32, device=device)
        self.pool = torch.cuda.graph_pool_handle()
        self.stream = torch.cuda.Stream(device)
        self.flat = torch.zeros(flat_capacity, dtype=torch.uint8, device=device)
        self.captures = 0
        self.replays = 0
        self.eager_steps = 0
        # data parallel (FlatMaster world > 1): the bucketed gradient all-reduces are captured
        # with the step on either route -- RCCL collectives (its graph-capture support: the
        # communicator's kernels become graph nodes on its internal stream, joined back by
        # events) or the xGMI kernel (device-side barrier epochs: replay-safe)
        self.capturable = True
        # MXTRAIN_GRAPH_DEBUG=1: synchronise after every step and log capture/replay events
        self.debug = os.environ.get("MXTRAIN_GRAPH_DEBUG", "0") == "1"
        self.marker = None   # diagnostics hook: called around the capture window
        self.graph_info: Dict[tuple, dict] = {}   # per captured shape: node census
        self.ctrl = self._control_group() if (flat_master is not None and flat_master.world > 1) else None
        self.handshakes = 0
        self.regrows = 0

    def _control_group(self):
        """Host-side control plane for the capture / capacity agreement: the data group
        itself when it is gloo, else a gloo group over the same ranks (collective call:
        every rank constructs its GraphedTrainStep at the same point)."""
        import torch.distributed as dist
        g = self.fm.group
        if dist.get_backend(g) == "gloo":
            return g
        return dist.new_group(ranks=dist.get_process_group_ranks(g), backend="gloo")

    def _agree(self, vals: List[int], op=None) -> List[int]:
        import torch.distributed as dist
        t = torch.tensor(vals, dtype=torch.int64)
        dist.all_reduce(t, op=op or dist.ReduceOp.MAX, group=self.ctrl)
        return [int(v) for v in t.tolist()]

    def _dbg(self, what: str, key) -> None:
        if self.debug:
            torch.cuda.synchronize(self.device)
            print(f"[graphed] {what} key={key} captures={self.captures} replays={self.replays} "
                  f"graphs={len(self.graphs)}", file=sys.stderr, flush=True)

    def _body(self, st: Dict[str, torch.Tensor]) -> torch.Tensor:
        losses = self.model(st["images"], st["hw"], st["gt_boxes"], st["gt_labels"], st["gt_count"], self.flat,
                            st["gt_mask_table"])
        losses["total_loss"].backward()
        if self.fm is not None:
            self.fm.step()
        else:
            if self.clip > 0:
                torch.nn.utils.clip_grad_norm_(self.params, self.clip, foreach=True)
            sgd_momentum_(self.opt, self.lr)
        return torch.stack([losses[k].detach().float() for k in LOSS_NAMES])

    def _eager(self, batch) -> Dict[str, torch.Tensor]:
        """The same step without a graph (after a failed capture)."""
        flat = batch["gt_mask_flat"]
        st = {k: batch[k].to(self.device, non_blocking=True) for k in INPUT_KEYS}
        self.flat[:flat.numel()].copy_(flat, non_blocking=True)
        self.opt.zero_grad(set_to_none=True)
        out = self._body(st)
        self.eager_steps += 1
        return dict(zip(LOSS_NAMES, out.unbind(0)))

    def _ensure_capacity(self, n: int) -> None:
        """Grow the mask buffer to hold ``n`` bytes (data parallel: ``n`` is already the
        MAX over ranks, so every rank grows -- and recaptures -- on the same step)."""
        if n <= self.flat.numel():
            return
        cap = self.flat.numel()
        while cap < n:
            cap *= 2
        # the graphs read the old buffer's address: drop them (recaptured on next use)
        self._drop_graphs()
        self.regrows += 1
        self.flat = torch.zeros(cap, dtype=torch.uint8, device=self.device)

    def _drop_graphs(self) -> None:
        self.graphs.clear()

    def _finish_capture(self, g, key) -> None:
        """Between capture and instantiation: memset nodes (MIOpen zeroes its accumulation
        workspaces and index buffers with hipMemsetAsync) replay wrong under the runtime's
        graph packet capture -- the cause of this step's illegal-address fault after a few
        replays (csrc/graph.hip) -- so they become fill-kernel nodes; the node census before
        the rewrite is kept for diagnostics."""
        from mxtrain.runtime import graphfix
        info = {"nodes": graphfix.census(g)}
        info["memsets_as_kernels"] = graphfix.memsets_to_kernels(g)
        self.graph_info[key] = info
        g.instantiate()

    def __call__(self, batch: Dict[str, torch.Tensor], lr: float) -> Dict[str, torch.Tensor]:
        flat = batch["gt_mask_flat"]
        key = tuple(tuple(batch[k].shape) for k in INPUT_KEYS)
        need_bytes, any_need = flat.numel(), 0
        if self.ctrl is not None and self.capturable:
            # collective: [anyone needs a capture, largest mask payload]
            need = int(self.capturable and (key not in self.graphs or need_bytes > self.flat.numel()))
            any_need, need_bytes = self._agree([need, need_bytes])
            self.handshakes += 1
        self._ensure_capacity(need_bytes)
        cur = torch.cuda.current_stream(self.device)
        self.lr.fill_(lr)
        entry = self.graphs.get(key)
        if not self.capturable:
            return self._eager(batch)
        if self.ctrl is not None and any_need:
            # capture round: the ranks that meet a new shape capture it, the others run the
            # same step eagerly (the same collectives); then all agree on the outcome
            if entry is None:
                out, err = self._capture(batch, key, cur)
            else:
                out, err = self._eager(batch), None
            import torch.distributed as dist
            if self._agree([0 if err else 1], op=dist.ReduceOp.MIN)[0] == 0:
                self._give_up(err or "capture failed on another rank")
            return out
        if entry is None:
            out, err = self._capture(batch, key, cur)
            if err is not None:
                self._give_up(err)
            return out
        g, st, sout = entry
        for k in INPUT_KEYS:
            st[k].copy_(batch[k], non_blocking=True)
        self.flat[:flat.numel()].copy_(flat, non_blocking=True)
        g.replay()
        self.replays += 1
        self._dbg("replayed", key)
        # the pool is shared: copy the losses out before another graph can reuse it
        return dict(zip(LOSS_NAMES, sout.clone().unbind(0)))

    def _capture(self, batch, key, cur):
        """Eager step + capture of this shape -> (losses of the eager step, error or None)."""
        flat = batch["gt_mask_flat"]
        st = {k: batch[k].to(self.device, non_blocking=True) for k in INPUT_KEYS}
        self.flat[:flat.numel()].copy_(flat, non_blocking=True)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            # eager step with this batch (a real update): warms every lazy cache
            self.opt.zero_grad(set_to_none=True)
            out = self._body(st)
            # capture: grads are allocated inside the graph's pool, never zeroed
            self.opt.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph(keep_graph=True)
            if self.marker is not None:
                torch.cuda.synchronize(self.device)
                self.marker("capture-begin")
            err = None
            try:
                # thread-local capture mode: the loader's threads keep pinning and copying host
                # buffers while this thread captures; under the default global mode such a
                # call from ANY thread invalidates the capture (seen at 4 img/GPU once the
                # fused stem shortened the forward: hipErrorStreamCaptureInvalidated)
                with torch.cuda.graph(g, pool=self.pool, stream=self.stream, capture_error_mode="thread_local"):
                    sout = self._body(st)
                if self.marker is not None:
                    self.marker("capture-end")
                self._finish_capture(g, key)
            except Exception as e:  # noqa: BLE001 -- fall back to the eager step, loudly
                err = repr(e)[:300]
                if self.debug:
                    import traceback
                    traceback.print_exc()
        cur.wait_stream(self.stream)
        res = dict(zip(LOSS_NAMES, out.unbind(0)))
        if err is not None:
            self.eager_steps += 1
            return res, err
        self.graphs[key] = (g, st, sout)
        self.captures += 1
        self._dbg("captured", key)
        if self.debug:
            print(f"[graphed] graph {key}: {self.graph_info[key]}", file=sys.stderr, flush=True)
        return res, None

    def _give_up(self, err: str) -> None:
        """Train eagerly from now on (every rank together: the caller agreed on it)."""
        print(f"[graphed] capture failed, training eagerly: {err}", file=sys.stderr, flush=True)
        self.capturable = False
        self._drop_graphs()

"""Batched fp32 -> bf16 compute copies of a model's trainable weights (AMP-style master
weights without one cast kernel per tensor).

The detection model keeps fp32 parameters (the optimizer, Horovod all-reduce and the
tensorpack checkpoint contract see fp32) and computes in bf16.  Casting every weight
inside its module's forward costs ~2 kernels per tensor forward (cast, plus the FrozenBN
scale multiply of a folded conv) and ~2 in backward -- about 300 launches and their
Python dispatch per Mask R-CNN step, most of them a few microseconds long.  Here ONE
autograd Function produces all compute copies with multi-tensor ``_foreach`` kernels
(fold-scale multiply, then cast into one flat bf16 buffer) and its backward returns all
fp32 gradients the same way; the modules look their copy up with ``cw(param, dtype)``.

    with ComputeWeights(model.compute_weight_specs(), torch.bfloat16):
        losses = model(...)            # modules call cw(p, dt) / folded convs call cw(w)

Gradients reach the fp32 parameters through the Function, so optimizers, clipping and
gradient hooks are unchanged.  Under data parallelism the specs are cut into ``groups``
contiguous node groups (model order): a group's fp32 gradients -- and so its DDP / Horovod
bucket hooks -- become ready as soon as backward has passed the first module that uses
it, instead of all at the very end of backward, so the gradient all-reduce overlaps the
rest of backward again.  Frozen parameters (requires_grad False) are not
included: their modules keep caching their own copies (resnet.ConvNorm._folded).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence, Tuple

import torch

_ACTIVE: Dict[int, torch.Tensor] = {}


def cw(p: torch.Tensor, dt: torch.dtype) -> torch.Tensor:
    """The active compute copy of parameter ``p`` (already scaled when it was registered
    with a fold scale), else a plain cast."""
    t = _ACTIVE.get(id(p))
    if t is not None:
        return t
    return p.to(dt)


def has(p: torch.Tensor) -> bool:
    return id(p) in _ACTIVE


class _CastAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dt, scales, scaled_idx, *params):
        ctx.scales, ctx.scaled_idx = scales, scaled_idx
        src = list(params)
        if scaled_idx:
            prod = torch._foreach_mul([params[i] for i in scaled_idx], [scales[i] for i in scaled_idx])
            for i, t in zip(scaled_idx, prod):
                src[i] = t
        sizes = [p.numel() for p in params]
        flat = torch.empty(sum(sizes), dtype=dt, device=params[0].device)
        outs = []
        for v, p in zip(flat.split(sizes), params):
            if p.dim() == 4:
                # conv weights in channels_last, the layout MIOpen's NHWC kernels take,
                # so the conv does not transpose the weight on every call
                o, i, kh, kw = p.shape
                outs.append(v.view(o, kh, kw, i).permute(0, 3, 1, 2))
            else:
                outs.append(v.view(p.shape))
        torch._foreach_copy_(outs, src)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        idx = [i for i, g in enumerate(grads) if g is not None]
        out: List[Optional[torch.Tensor]] = [None] * len(grads)
        if idx:
            g32 = [torch.empty(grads[i].shape, dtype=torch.float32, device=grads[i].device) for i in idx]
            torch._foreach_copy_(g32, [grads[i] for i in idx])
            pos = {i: j for j, i in enumerate(idx)}
            sc = [i for i in ctx.scaled_idx if i in pos]
            if sc:
                # d(w * s)/dw = s
                torch._foreach_mul_([g32[pos[i]] for i in sc], [ctx.scales[i] for i in sc])
            for i, g in zip(idx, g32):
                out[i] = g
        return (None, None, None, *out)


class ComputeWeights:
    """Context manager: builds the compute copies of ``specs`` = [(param, fold_scale or
    None)] once on entry (one autograd node) and makes them visible to cw()."""

    def __init__(self, specs: Sequence[Tuple[torch.Tensor, Optional[torch.Tensor]]], dt: torch.dtype,
                 groups: int = 1):
        self.specs = [(p, s) for p, s in specs if p.requires_grad]
        self.dt = dt
        self.groups = max(1, int(groups))

    @staticmethod
    def split(specs, groups: int):
        """Contiguous chunks of ~equal parameter count (model order kept)."""
        if groups <= 1 or len(specs) <= 1:
            return [list(specs)]
        total = sum(p.numel() for p, _ in specs)
        out, cur, acc = [], [], 0
        for p, s in specs:
            cur.append((p, s))
            acc += p.numel()
            if acc >= total * (len(out) + 1) / groups and len(out) < groups - 1:
                out.append(cur)
                cur = []
        if cur:
            out.append(cur)
        return out

    def __enter__(self):
        if self.specs and torch.is_grad_enabled():
            for chunk in self.split(self.specs, self.groups):
                params = [p for p, _ in chunk]
                scales = [s for _, s in chunk]
                scaled = [i for i, s in enumerate(scales) if s is not None]
                outs = _CastAll.apply(self.dt, scales, scaled, *params)
                for p, o in zip(params, outs):
                    _ACTIVE[id(p)] = o
        return self

    def __exit__(self, *exc):
        for p, _ in self.specs:
            _ACTIVE.pop(id(p), None)
        return False


def _cast_dense(t: torch.Tensor) -> bool:
    return (t.is_cuda and t.numel() % 8 == 0 and t.data_ptr() % 16 == 0
            and (t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))))


def _cast_launch(pairs, to_bf16: bool) -> None:
    """One csrc/cast.hip launch per <= 96 (src, dst) pairs of equal memory order."""
    from ..ops import _lib
    for i in range(0, len(pairs), 96):
        chunk = pairs[i:i + 96]
        d = ctypes_int64_array([v for s, t in chunk for v in (s.data_ptr(), t.data_ptr(), s.numel())])
        _lib.call("mx_cast_multi", d, len(chunk), int(to_bf16), _lib.stream())


class _CastGroup(torch.autograd.Function):
    """bf16 compute copies of fp32 weights in ONE launch (csrc/cast.hip), each copy with its
    weight's strides; the backward casts their bf16 gradients to fp32 in one launch too
    (gradients in another memory order fall back to a plain cast).  ``state`` (a dict shared
    by the groups of one forward): ``left`` groups whose backward has not run -- the
    implicit-GEMM weight gradients' deferred split-K reductions (ops/convwg.py) are flushed
    before each group's cast, deferral staying on while groups remain."""

    @staticmethod
    def forward(ctx, state, *params):
        sizes = [p.numel() for p in params]
        flat = torch.empty(sum(sizes), dtype=torch.bfloat16, device=params[0].device)
        outs, off = [], 0
        for p, n in zip(params, sizes):
            outs.append(flat[off:off + n].as_strided(p.shape, p.stride()))
            off += n
        _cast_launch(list(zip(params, outs)), True)
        ctx.meta = [(p.shape, p.stride()) for p in params]
        ctx.state = state
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        st = ctx.state
        if st is not None and st.get("defer"):
            from ..ops import convwg
            st["left"] -= 1
            convwg.defer_flush(keep_on=st["left"] > 0)
        out: List[Optional[torch.Tensor]] = [None] * len(grads)
        pairs = []
        for i, g in enumerate(grads):
            if g is None:
                continue
            shape, stride = ctx.meta[i]
            if g.stride() == stride and _cast_dense(g):
                out[i] = torch.empty_strided(shape, stride, dtype=torch.float32, device=g.device)
                pairs.append((g, out[i]))
            else:
                out[i] = torch.empty_strided(shape, stride, dtype=torch.float32, device=g.device).copy_(g)
        if pairs:
            _cast_launch(pairs, False)
        return (None,) + tuple(out)


class CastGroup:
    """Context manager: bf16 compute copies of ``params`` (fp32, dense, numel % 8 == 0) from
    one launch per group, visible to cw() -- the one-launch form of per-module weight casts
    under bf16 autocast.  ``groups`` > 1 cuts them into contiguous chunks (data parallel:
    their fp32 gradients, and DDP's bucket hooks, then become ready during backward)."""

    # the split-K weight-gradient reductions of the convolutions using these copies run as one
    # batched launch per group backward (ops/convwg.py defer_begin / defer_flush) instead of
    # one launch per convolution (44 per ResNet-50 step)
    # (44 launches / 427 us -> 2 / 283 us per step; launcher A/B within noise:
    # profiles/r6/resnet_launcher_ab_deferred_wgrad_reduce.txt)
    DEFER = True

    def __init__(self, params, groups: int = 1):
        self.params = [p for p in params if p.requires_grad and _cast_dense(p) and p.dtype == torch.float32]
        self.groups = max(1, int(groups))

    def __enter__(self):
        if self.params and torch.is_grad_enabled():
            chunks = ComputeWeights.split([(p, None) for p in self.params], self.groups)
            defer = CastGroup.DEFER and self.params[0].is_cuda
            state = {"left": len(chunks), "defer": defer}
            keys = []
            for chunk in chunks:
                ps = [p for p, _ in chunk]
                for p, o in zip(ps, _CastGroup.apply(state, *ps)):
                    _ACTIVE[id(p)] = o
                    keys.append(o.data_ptr())
            if defer:
                from ..ops import convwg
                convwg.defer_begin(keys)
        return self

    def __exit__(self, *exc):
        for p in self.params:
            _ACTIVE.pop(id(p), None)
        return False


# ------------------------------------------------------------------------- flat master
def _align8(n: int) -> int:
    return (n + 7) // 8 * 8


def _align(n: int, a: int) -> int:
    return (n + a - 1) // a * a


class _FlatCast(torch.autograd.Function):
    """Forward: the FlatMaster's persistent compute copies of one bucket (refreshed by the
    optimizer pass, re-cast only when stale); backward: the bucket's gradients into the flat
    fp32 buffer in one launch (returned as views of it) -- and, data-parallel, that slice's
    all-reduce is started right away, while backward continues with earlier layers."""

    @staticmethod
    def forward(ctx, fm, k, *params):
        ctx.fm, ctx.k = fm, k
        fm.ensure_fresh()
        tb, te = fm.buckets[k][:2]
        return tuple(fm.compute_views()[tb:te])

    @staticmethod
    def backward(ctx, *grads):
        return (None, None, *ctx.fm.grads_in(grads, ctx.k))


class FlatMaster:
    """Flat fp32 master weights, gradients and SGD momentum for a single-process training
    loop, plus persistent bf16 compute copies (folded FrozenBN scale applied, conv weights
    channels_last) written by the optimizer pass itself (csrc/multitensor.hip):

        forward   no cast kernels (the copies are current)
        backward  1 launch: bf16 grads -> flat fp32 grads (x fold scale) + sum-of-squares
                  partials, 1 launch: ||g||^2
        optimizer 1 launch: clip + SGD momentum + compute-copy refresh

    torch.optim.SGD semantics (dampening 0, no Nesterov, per-group weight decay) and
    torch.nn.utils.clip_grad_norm_'s coefficient; the SGD instance keeps its param groups
    and its momentum buffers (views of the flat buffer), so state_dict() and checkpoints
    are unchanged (call ``rebind_state()`` after ``opt.load_state_dict``).  Parameters
    become views of the flat buffer (``p.data``), so in-place writes (checkpoint load)
    land in it and bump the versions that mark the copies stale.

    Data parallel (``group`` with world > 1; the reference's Horovod Mask R-CNN runs,
    examples/maskrcnn/train-maskrcnn-tensorpack.yaml:34, mpijob-horovod values.yaml:64-66):
    parameters are laid out in model order and cut into ~``bucket_bytes`` buckets, one
    autograd node each.  When backward has produced a bucket's gradients (the heads first,
    the backbone stem last) its flat fp32 slice is all-reduced at once -- RCCL
    asynchronously, or the direct xGMI kernel (parallel/xgmi.py, MXTRAIN_XGMI) on a side
    stream -- in a fixed bucket order on every rank.  ``step()`` joins them, averages and
    takes ||g||^2 of the averaged gradient in one pass (clip as Horovod + clip_grad_norm_),
    then runs the same fused clip + SGD launch.  Every piece is capturable, so the whole
    data-parallel step can be one hipGraph.
    """

    def __init__(self, model, opt: torch.optim.SGD, clip: float, dt: torch.dtype = torch.bfloat16,
                 group=None, bucket_bytes: int = 32 << 20, force_dp: bool = False):
        from ..ops import _lib
        self.model, self.opt, self.dt = model, opt, dt
        mom = {g["momentum"] for g in opt.param_groups}
        wds = {float(g["weight_decay"]) for g in opt.param_groups} - {0.0}
        assert len(mom) == 1 and len(wds) <= 1, "one momentum and one non-zero weight decay"
        assert all(not g.get("nesterov") and not g.get("dampening") for g in opt.param_groups)
        import torch.distributed as dist
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist_on else 1
        # an explicit group object: the xGMI communicator registry is keyed on it
        self.group = group if (group is not None or not dist_on) else dist.group.WORLD
        # the data-parallel machinery (buckets, per-bucket all-reduce, joined average) runs
        # when world > 1; ``force_dp`` runs it on a one-rank group too (tests: the RCCL
        # all-reduce captured inside the step graph on one GPU)
        self.dp = self.world > 1 or (bool(force_dp) and dist_on)
        self.params, wdf = [], []
        for g in opt.param_groups:
            for p in g["params"]:
                if p.requires_grad:
                    self.params.append(p)
                    wdf.append(1 if g["weight_decay"] else 0)
        if self.dp:
            # model order: backward finishes the last modules' gradients first
            order = {id(p): i for i, p in enumerate(model.parameters())}
            pairs = sorted(zip(self.params, wdf), key=lambda pw: order.get(id(pw[0]), len(order)))
            self.params, wdf = [p for p, _ in pairs], [w for _, w in pairs]
        dev = self.params[0].device
        self.device = dev
        self.cuda = dev.type == "cuda"
        self.chunk = _lib.query("mx_mt_chunk") if self.cuda else 2048
        self.sizes = [p.numel() for p in self.params]
        # buckets (tensor range, flat element range); bucket slices start 64-element
        # (256-B) aligned so every all-reduce message divides over 8 ranks in 16-B units
        self.offs, off = [], 0
        self.buckets: List[Tuple[int, int, int, int]] = []
        cap = max(1, bucket_bytes // 4) if self.dp else None
        tb, e0 = 0, 0
        for t, n in enumerate(self.sizes):
            self.offs.append(off)
            off += _align8(n)
            if cap is not None and off - e0 >= cap and t + 1 < len(self.sizes):
                off = _align(off, 64)
                self.buckets.append((tb, t + 1, e0, off))
                tb, e0 = t + 1, off
        if cap is not None:
            off = _align(max(off, 8), 64)
        self.buckets.append((tb, len(self.sizes), e0, max(off, 8)))
        total = max(off, 8)
        # layout: 4-D (conv) weights channels_last [d0, kh, kw, d1] in the fp32 buffers too,
        # i.e. the bf16 copy's order, so every multi-tensor pass (gradient in, SGD + copy out)
        # is a linear vector stream; the parameters are channels_last-strided views of it
        self.geo = []
        for p in self.params:
            s = p.shape
            d0 = s[0] if p.dim() >= 1 else 1
            d1 = s[1] if p.dim() >= 2 else 1
            inner = int(torch.Size(s[2:]).numel()) if p.dim() >= 3 else 1
            self.geo.append((d0, d1, inner, 1 if p.dim() == 4 else 0))
        self.P = torch.zeros(total, dtype=torch.float32, device=dev)
        self.G = torch.zeros(total, dtype=torch.float32, device=dev)
        self.M = torch.zeros(total, dtype=torch.float32, device=dev)
        self.W = torch.zeros(total, dtype=dt, device=dev)
        with torch.no_grad():
            for t, p in enumerate(self.params):
                v = self._fview(self.P, t)
                v.copy_(p.detach())
                p.data = v
        self.rebind_state()
        nb = [(n + self.chunk - 1) // self.chunk for n in self.sizes]
        self.bstart_host = [0]
        for k in nb:
            self.bstart_host.append(self.bstart_host[-1] + k)
        self.nblocks = self.bstart_host[-1]
        bmap = [t for t, k in enumerate(nb) for _ in range(k)]
        self.bmap = torch.tensor(bmap or [0], dtype=torch.int32, device=dev)
        self.bstart = torch.tensor(self.bstart_host, dtype=torch.int32, device=dev)
        self._bstart_arr = ctypes_int_array(self.bstart_host)   # kept alive: its address is passed
        self.bstart_c = ctypes.addressof(self._bstart_arr)
        self.wdf = wdf
        self.scales: List[Optional[torch.Tensor]] = [None] * len(self.params)
        self._scale_key = None
        self.tab = torch.zeros(len(self.params), 8, dtype=torch.int64, device=dev)
        self.hyper = torch.zeros(4, dtype=torch.float32, device=dev)
        self.hyper[1] = float(mom.pop())
        self.hyper[2] = float(wds.pop()) if wds else 0.0
        self.hyper[3] = float(clip or 0.0)
        self.lr = self.hyper[0:1].view(())   # device scalar: fill_ before a (graph) step
        self.normsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.partial = torch.zeros(max(self.nblocks, (total + self.chunk - 1) // self.chunk, 1), dtype=torch.float32,
                                   device=dev)
        self.zero_bf16 = torch.zeros(_align8(max(self.sizes)), dtype=dt, device=dev)
        self._wkey = None
        self._cw_specs = None
        self._dp_stream = torch.cuda.Stream(device=dev) if (self.cuda and self.dp) else None
        self.dp_route = None     # route of the last bucket reduced: "xgmi" / "rccl" / "gloo"
        self.dp_routes = set()   # every route used so far
        self._dp_reset()

    def _fview(self, buf: torch.Tensor, t: int) -> torch.Tensor:
        """Parameter t's slice of a flat fp32 buffer as a tensor of the parameter's shape
        (channels_last-strided for 4-D weights: the buffer holds them in [d0, kh, kw, d1] order)."""
        p, o, n = self.params[t], self.offs[t], self.sizes[t]
        d0, d1, inner, cl = self.geo[t]
        v = buf[o:o + n]
        if cl and inner > 1:
            return v.view(d0, p.shape[2], p.shape[3], d1).permute(0, 3, 1, 2)
        return v.view(p.shape)

    # -------------------------------------------------------------- optimizer state
    def rebind_state(self) -> None:
        """Momentum buffers as views of the flat buffer (after construction or after
        ``opt.load_state_dict``, which installs fresh tensors)."""
        with torch.no_grad():
            for t, p in enumerate(self.params):
                st = self.opt.state[p]
                buf = st.get("momentum_buffer")
                view = self._fview(self.M, t)
                if buf is not None and buf.data_ptr() != view.data_ptr():
                    view.copy_(buf)
                st["momentum_buffer"] = view

    # -------------------------------------------------------------- fold scales
    def refresh_scales(self) -> None:
        specs = self.model.compute_weight_specs()
        if specs is self._cw_specs:
            return
        self._cw_specs = specs
        full = {id(p): s for p, s in specs}
        scales = []
        for p, (d0, _, _, _) in zip(self.params, self.geo):
            s = full.get(id(p))
            scales.append(None if s is None else s.reshape(d0, -1)[:, 0].float().contiguous())
        self.scales = scales
        rows = []
        for t, (p, o, n) in enumerate(zip(self.params, self.offs, self.sizes)):
            d0, d1, inner, cl = self.geo[t]
            sp = scales[t].data_ptr() if (scales[t] is not None and self.cuda) else 0
            # cl = 0 for the kernels: the fp32 buffers already hold the copy's order
            rows.append([o, n, d0, d1, inner, 0, sp, self.wdf[t]])
        self.tab.copy_(torch.tensor(rows, dtype=torch.int64))
        self._scale_key = object()   # new identity: the copies must be re-cast

    def _key(self):
        return (tuple(p._version for p in self.params), self._scale_key)

    # -------------------------------------------------------------- compute copies
    def compute_views(self) -> List[torch.Tensor]:
        outs = []
        for p, o, n, (d0, d1, inner, cl) in zip(self.params, self.offs, self.sizes, self.geo):
            v = self.W[o:o + n]
            if cl:
                kh, kw = p.shape[2], p.shape[3]
                outs.append(v.view(d0, kh, kw, d1).permute(0, 3, 1, 2))
            else:
                outs.append(v.view(p.shape))
        return outs

    def ensure_fresh(self) -> None:
        self.refresh_scales()
        key = self._key()
        if key == self._wkey:
            return
        if self.cuda:
            from ..ops import _lib
            _lib.call("mx_mt_cast", self.tab.data_ptr(), self.bmap.data_ptr(), self.bstart.data_ptr(),
                      self.nblocks, self.P.data_ptr(), self.W.data_ptr(), _lib.stream())
        else:
            with torch.no_grad():
                for p, v, s in zip(self.params, self.compute_views(), self.scales):
                    w = p.detach() if s is None else p.detach() * s.view(-1, *([1] * (p.dim() - 1)))
                    v.copy_(w)
        self._wkey = key

    def compute_weights(self):
        """Context manager registering the compute copies for ``cw()`` (one autograd
        node; under no_grad the copies are plain views)."""
        fm = self

        class _Ctx:
            def __enter__(self_):
                if torch.is_grad_enabled():
                    fm._dp_reset()
                    outs = []
                    for k, (tb, te, _, _) in enumerate(fm.buckets):
                        outs.extend(_FlatCast.apply(fm, k, *fm.params[tb:te]))
                    if fm.cuda:   # the step's weight-gradient reductions: one launch
                        from ..ops import convwg
                        convwg.defer_begin([o.data_ptr() for o in outs])
                else:
                    fm.ensure_fresh()
                    outs = fm.compute_views()
                for p, o in zip(fm.params, outs):
                    _ACTIVE[id(p)] = o
                return self_

            def __exit__(self_, *exc):
                for p in fm.params:
                    _ACTIVE.pop(id(p), None)
                return False
        return _Ctx()

    # -------------------------------------------------------------- backward / step
    def grads_in(self, grads, k: int = 0) -> List[torch.Tensor]:
        """Gradients of bucket k's compute copies (bf16, copy layout; None = no gradient)
        -> its slice of the flat fp32 buffer (x fold scale), with sum-of-squares partials."""
        tb, te, _, _ = self.buckets[k]
        if self.cuda:
            from ..ops import convwg
            convwg.defer_flush(keep_on=self.dp and len(self._ready) + 1 < len(self.buckets))
        srcs = []
        keep = []
        for t, g in zip(range(tb, te), grads):
            d0, d1, inner, cl = self.geo[t]
            if g is None:
                srcs.append(None)
                continue
            if cl and inner > 1:
                if not g.is_contiguous(memory_format=torch.channels_last):
                    g = g.contiguous(memory_format=torch.channels_last)
            elif not g.is_contiguous() and not (cl and g.is_contiguous(memory_format=torch.channels_last)):
                g = g.contiguous()
            if g.dtype != self.dt:
                g = g.to(self.dt)
            if self.cuda and g.data_ptr() % 16:
                g = g.clone(memory_format=torch.channels_last if (cl and inner > 1) else torch.contiguous_format)
            keep.append(g)
            srcs.append(g)
        if self.cuda:
            from ..ops import _lib
            ptrs = [(s.data_ptr() if s is not None else self.zero_bf16.data_ptr()) for s in srcs]
            arr = ctypes_int64_array(ptrs)
            _lib.call("mx_mt_grad_in_range", self.tab.data_ptr(), self.bmap.data_ptr(), self.bstart.data_ptr(),
                      self.bstart_c, tb, te, ctypes.addressof(arr), self.G.data_ptr(), self.partial.data_ptr(),
                      _lib.stream())
            if not self.dp:
                _lib.call("mx_mt_sumsq_fin", self.partial.data_ptr(), self.nblocks, self.normsq.data_ptr(),
                          _lib.stream())
        else:
            with torch.no_grad():
                acc = torch.zeros((), dtype=torch.float32)
                for t, s in zip(range(tb, te), srcs):
                    p = self.params[t]
                    gv = torch.zeros(p.shape) if s is None else s.float()
                    if self.scales[t] is not None:
                        gv = gv * self.scales[t].view(-1, *([1] * (p.dim() - 1)))
                    self._fview(self.G, t).copy_(gv)
                    acc = acc + gv.pow(2).sum()
                if not self.dp:
                    self.normsq.fill_(float(acc))
        if self.dp:
            self._dp_ready(k)
        return [self._fview(self.G, t) for t in range(tb, te)]

    # -------------------------------------------------------------- data parallel
    def _dp_reset(self) -> None:
        self._ready = set()
        self._next = len(self.buckets) - 1   # buckets are reduced last-to-first on every rank
        self._works = []
        self._side_used = False

    def _dp_ready(self, k: int) -> None:
        self._ready.add(k)
        while self._next >= 0 and self._next in self._ready:
            self._reduce_bucket(self._next)
            self._next -= 1

    def _reduce_bucket(self, k: int) -> None:
        import torch.distributed as dist
        _, _, e0, e1 = self.buckets[k]
        seg = self.G[e0:e1]
        if self.cuda:
            from ..parallel import xgmi
            comm = xgmi.route(self.group, seg, "all_reduce", seg.numel() * 4)
            if comm is not None:
                cur = torch.cuda.current_stream(self.device)
                self._dp_stream.wait_stream(cur)
                with torch.cuda.stream(self._dp_stream):
                    comm.all_reduce_(seg)
                self._side_used = True
                self.dp_route = "xgmi"
                self.dp_routes.add("xgmi")
                return
        self._works.append(dist.all_reduce(seg, group=self.group, async_op=True))
        self.dp_route = "rccl" if self.cuda else "gloo"
        self.dp_routes.add(self.dp_route)

    def finish_grads(self) -> None:
        """Data parallel: make sure every bucket was reduced (a bucket whose parameters
        got no gradient at all still contributes zeros), join the reductions, average and
        take ||g||^2 of the averaged gradient."""
        if not self.dp:
            return
        for k in range(self._next, -1, -1):
            if k not in self._ready:
                tb, te, _, _ = self.buckets[k]
                self.grads_in([None] * (te - tb), k)
        for w in self._works:
            w.wait()
        if self._side_used:
            torch.cuda.current_stream(self.device).wait_stream(self._dp_stream)
        if self.cuda:
            from ..ops import _lib
            n = self.buckets[-1][3]
            nparts = (n + self.chunk - 1) // self.chunk
            assert nparts <= self.partial.numel()
            _lib.call("mx_mt_scale_sumsq", self.G.data_ptr(), n, 1.0 / self.world, self.partial.data_ptr(),
                      _lib.stream())
            _lib.call("mx_mt_sumsq_fin", self.partial.data_ptr(), nparts, self.normsq.data_ptr(), _lib.stream())
        else:
            with torch.no_grad():
                self.G.mul_(1.0 / self.world)
                self.normsq.fill_(float(self.G.double().pow(2).sum()))
        self._dp_reset()

    def step(self, lr=None) -> None:
        """clip + SGD momentum + compute-copy refresh (lr: float, or None when the
        device scalar ``self.lr`` was filled already -- graph replay)."""
        if lr is not None:
            self.lr.fill_(float(lr))
        if self.cuda:   # every deferred reduction launched, deferral off until the next step
            from ..ops import convwg
            convwg.defer_flush(keep_on=False)
        self.finish_grads()
        if self.cuda:
            from ..ops import _lib
            _lib.call("mx_mt_sgd", self.tab.data_ptr(), self.bmap.data_ptr(), self.bstart.data_ptr(), self.nblocks,
                      self.P.data_ptr(), self.G.data_ptr(), self.M.data_ptr(), self.W.data_ptr(),
                      self.hyper.data_ptr(), self.normsq.data_ptr(), _lib.stream())
        else:
            with torch.no_grad():
                lr_, mom, wd, clip = (float(x) for x in self.hyper.tolist())
                cc = 1.0
                if clip > 0:
                    cc = min(1.0, clip / (float(self.normsq[0]) ** 0.5 + 1e-6))
                n_all = self.P.numel()
                wdv = torch.zeros(n_all)
                for t, (o, n) in enumerate(zip(self.offs, self.sizes)):
                    if self.wdf[t]:
                        wdv[o:o + n] = wd
                d = self.G * cc + wdv * self.P
                self.M.mul_(mom).add_(d)
                self.P.sub_(lr_ * self.M)
                for p, v, s in zip(self.params, self.compute_views(), self.scales):
                    w = p.detach() if s is None else p.detach() * s.view(-1, *([1] * (p.dim() - 1)))
                    v.copy_(w)
        self._wkey = self._key()


def ctypes_int64_array(vals):
    return (ctypes.c_int64 * len(vals))(*vals)


def ctypes_int_array(vals):
    return (ctypes.c_int * len(vals))(*vals)

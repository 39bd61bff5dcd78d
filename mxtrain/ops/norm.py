"""LayerNorm / RMSNorm and the fused bias-dropout-add + norm (BDA-norm) ops.

GPU tensors run the HIP kernels of ``csrc/norm.hip``; CPU tensors run the fp32 PyTorch
reference below (also the numerics oracle of ``tests/test_kernels_gpu.py``).
"""
from __future__ import annotations

import torch

from . import _lib
from .rng import keep_mask


def _seed_val(seed_t, salt):
    if seed_t is None:
        return 0
    return (int(seed_t.reshape(-1)[0].item()) + salt) & 0xFFFFFFFF


# ------------------------------------------------------------------ reference (CPU)
def _ref_norm(h32, gamma, beta, eps, rms):
    if rms:
        rstd = torch.rsqrt(h32.pow(2).mean(-1) + eps)
        mean = torch.zeros_like(rstd)
        y = h32 * rstd[:, None] * gamma.float()
    else:
        mean = h32.mean(-1)
        var = (h32 - mean[:, None]).pow(2).mean(-1)
        rstd = torch.rsqrt(var + eps)
        y = (h32 - mean[:, None]) * rstd[:, None] * gamma.float()
        if beta is not None:
            y = y + beta.float()
    return y, mean, rstd


def _ref_bda(x, bias, residual, p, seed_t, salt, elem0=0):
    t = x.float()
    if bias is not None:
        t = t + bias.float()
    if p > 0:
        m = keep_mask(t.numel(), _seed_val(seed_t, salt), p, base=elem0).view_as(t)
        t = torch.where(m, t / (1 - p), torch.zeros_like(t))
    if residual is not None:
        t = t + residual.float()
    return t


# ------------------------------------------------------------------ forward
def layernorm_fwd(x, gamma, beta, eps=1e-5, rms=False):
    """x [rows, cols] -> (y, mean, rstd)."""
    rows, cols = x.shape
    if not _lib.use_hip(x):
        y, mean, rstd = _ref_norm(x.float(), gamma, beta, eps, rms)
        return y.to(x.dtype), mean, rstd
    y = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    if rms:
        _lib.call("mx_rmsnorm_fwd", _lib.ptr(x), _lib.ptr(gamma), _lib.ptr(y), _lib.ptr(rstd),
                  rows, cols, eps, _lib.stream())
    else:
        _lib.call("mx_layernorm_fwd", _lib.ptr(x), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(y),
                  _lib.ptr(mean), _lib.ptr(rstd), rows, cols, eps, _lib.stream())
    return y, mean, rstd


def bda_norm_fwd(x, bias, residual, gamma, beta, eps=1e-5, p=0.0, seed_t=None, salt=0,
                 rms=False, *, elem0: int = 0):
    """h = residual + dropout(x + bias); y = norm(h).  Returns (h, y, mean, rstd).
    ``elem0``: flat index of x[0, 0] in the unsharded activation (the dropout mask is keyed
    on global element indices: a sequence-parallel shard draws the unsharded tensor's bits)."""
    rows, cols = x.shape
    if not _lib.use_hip(x):
        h32 = _ref_bda(x, bias, residual, p, seed_t, salt, elem0)
        h = h32.to(x.dtype)
        y, mean, rstd = _ref_norm(h.float(), gamma, beta, eps, rms)
        return h, y.to(x.dtype), mean, rstd
    h = torch.empty_like(x)
    y = torch.empty_like(x)
    mean = torch.empty(rows, dtype=torch.float32, device=x.device)
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    _lib.call("mx_bda_norm_fwd", _lib.ptr(x), _lib.ptr(bias), _lib.ptr(residual), _lib.ptr(gamma),
              _lib.ptr(beta), _lib.ptr(h), _lib.ptr(y), _lib.ptr(mean), _lib.ptr(rstd), rows, cols,
              eps, float(p), _lib.ptr(seed_t), salt, int(elem0), int(rms), _lib.stream())
    return h, y, mean, rstd


# ------------------------------------------------------------------ backward
def norm_bwd(dy, dres, h, mean, rstd, gamma, want_dx=False, p=0.0, seed_t=None, salt=0,
             rms=False, dgamma=None, dbeta=None, dbias=None, accumulate=False, defer=None, elem0: int = 0):
    """Backward of (bda_)norm.

    dh = dres + dnorm/dh;  dx = dh * dropout-mask * 1/(1-p) (if want_dx).
    Column reductions are written (or added when ``accumulate``) into the bf16 buffers
    ``dgamma``, ``dbeta``, ``dbias`` when given.  Returns (dh, dx or None).
    """
    rows, cols = dy.shape
    if not _lib.use_hip(dy):
        h32 = h.float()
        xh = (h32 - mean[:, None]) * rstd[:, None] if not rms else h32 * rstd[:, None]
        d32 = dy.float()
        gy = d32 * gamma.float()
        m1 = gy.mean(-1, keepdim=True) if not rms else 0.0
        m2 = (gy * xh).mean(-1, keepdim=True)
        dh32 = rstd[:, None] * (gy - m1 - xh * m2)
        if dres is not None:
            dh32 = dh32 + dres.float()
        dh = dh32.to(dy.dtype)
        dx = None
        if want_dx:
            t = dh.float()
            if p > 0:
                m = keep_mask(t.numel(), _seed_val(seed_t, salt), p, base=elem0).view_as(t)
                t = torch.where(m, t / (1 - p), torch.zeros_like(t))
            dx = t.to(dy.dtype)
        for buf, val in ((dgamma, (d32 * xh).sum(0)), (dbeta, d32.sum(0)),
                         (dbias, dx.float().sum(0) if dx is not None else None)):
            if buf is not None and val is not None:
                if accumulate:
                    buf.copy_((buf.float() + val).to(buf.dtype))
                else:
                    buf.copy_(val.to(buf.dtype))
        return dh, dx
    nparts = _lib.query("mx_norm_bwd_nparts2", rows, cols)
    outs = (dgamma, dbeta, dbias if want_dx else None)
    want = any(t is not None for t in outs)
    partial = None
    if defer is not None and want:
        partial = defer.partial(tuple(t.data_ptr() if t is not None else 0 for t in outs), outs, nparts,
                                3 * cols, 3, cols, accumulate)
    deferred = partial is not None
    if partial is None:
        scratch_n = _lib.query64("mx_colreduce_scratch", nparts, 3 * cols)
        partial = torch.empty(nparts * 3 * cols + scratch_n, dtype=torch.float32, device=dy.device)
    dh = torch.empty_like(dy)
    dx = torch.empty_like(dy) if want_dx else None
    _lib.call("mx_norm_bwd", _lib.ptr(dy), _lib.ptr(dres), _lib.ptr(h), _lib.ptr(mean),
              _lib.ptr(rstd), _lib.ptr(gamma), _lib.ptr(dh), _lib.ptr(dx), _lib.ptr(partial),
              rows, cols, float(p), _lib.ptr(seed_t), salt, int(elem0), int(rms), _lib.stream())
    if want and not deferred:
        scratch = partial[nparts * 3 * cols:]
        _lib.call("mx_colsum_finalize", _lib.ptr(partial), nparts, cols, 3, _lib.ptr(dgamma),
                  _lib.ptr(dbeta), _lib.ptr(dbias if want_dx else None), int(accumulate),
                  _lib.ptr(scratch), _lib.stream())
    return dh, dx


def colsum(x, out, accumulate=False, defer=None):
    """out (bf16 [cols]) (+)= x.sum(0) for x [rows, cols] bf16 (``defer``: partials now,
    reduction in the step's batched flush)."""
    rows, cols = x.shape
    if not _lib.use_hip(x):
        v = x.float().sum(0)
        if accumulate:
            v = v + out.float()
        out.copy_(v.to(out.dtype))
        return out
    nparts = (rows + 15) // 16
    if defer is not None:
        part = defer.partial((out.data_ptr(),), (out, None, None), nparts, cols, 1, cols, accumulate)
        if part is not None:
            _lib.call("mx_colsum_partial_bf16", _lib.ptr(x), rows, cols, _lib.ptr(part), _lib.stream())
            return out
    scratch_n = _lib.query64("mx_colreduce_scratch", nparts, cols)
    partial = torch.empty(nparts * cols + scratch_n, dtype=torch.float32, device=x.device)
    _lib.call("mx_colsum_bf16", _lib.ptr(x), rows, cols, _lib.ptr(partial), _lib.ptr(out),
              int(accumulate), _lib.stream())
    return out


def colsum_partials_buffer(nparts: int, cols: int, device):
    """fp32 buffer for nparts x cols column partials plus the immediate reduction's scratch;
    returns (partials view [nparts, cols], whole buffer)."""
    scratch_n = _lib.query64("mx_colreduce_scratch", nparts, cols)
    buf = torch.empty(nparts * cols + scratch_n, dtype=torch.float32, device=device)
    return buf[:nparts * cols].view(nparts, cols), buf


def colsum_finalize(buf, nparts: int, cols: int, out, accumulate=False):
    """out (bf16 [cols]) (+)= the column sums of the nparts x cols partials at the start of
    ``buf`` (from colsum_partials_buffer): the same deterministic reduction the deferred
    batched flush and colsum() use."""
    _lib.call("mx_colsum_finalize", _lib.ptr(buf), nparts, cols, 1, _lib.ptr(out), None, None,
              int(accumulate), _lib.ptr(buf) + 4 * nparts * cols, _lib.stream())
    return out


# ------------------------------------------------------------------ deferred column sums
class ColReduceQueue:
    """Column reductions of a training step deferred to ONE batched launch
    (``mx_colreduce_batched``) at the end of backward, instead of one colreduce launch per
    norm / bias-GeLU / bias producer (~100 per GPT-2 345M step).

    Every distinct output (LN dgamma/dbeta/dbias triple, bias gradient) owns a fixed region
    of a persistent fp32 arena holding the partials of all its producer calls of the step
    (micro-batches stacked), so the flush is one job per output -- a single accumulate
    into the bf16 gradient, no two jobs writing the same output.  The layout is recorded
    on the first step (which reduces immediately), then reused; a step whose producer
    sequence differs from the recorded one is an error (the step structure is static for a
    fixed model / batch configuration).

    Data parallel (``group_of``: output pointer -> gradient bucket): the jobs are split into
    one table per bucket and ``flush_group(b)`` reduces bucket b's outputs right before that
    bucket's reduce-scatter is issued (parallel/zero.py ``pre_reduce``) -- ~one launch per
    bucket instead of one per producer, and the gradients are final when they are
    communicated.  Outputs of one region must fall in one bucket, and no output may appear
    in two regions (two jobs would read-modify-write the same bf16 gradient); otherwise the
    queue stays in immediate mode."""

    def __init__(self, device, group_of=None):
        self.device = device
        self.group_of = group_of
        self.tables = {}        # group -> (table, njobs, nblocks)
        self.flushed = set()
        self.layout = None      # [(key, nparts, C, nvec, cols, accumulate)] in call order
        self.rec = []
        self.arena = None
        self.table = None
        self.regions = {}       # key -> (offset, rows_total, C, nvec, cols, outs, acc)
        self.i = 0
        self.active = False

    def begin(self):
        self.i = 0
        self.rec = []
        self.fill = {}
        self.flushed = set()
        self.active = self.layout is not None

    def partial(self, key, outs, nparts: int, C: int, nvec: int, cols: int, accumulate: bool):
        """fp32 [nparts * C] view for this producer's partials when deferred, else None
        (caller finalizes immediately; the call is recorded for the layout)."""
        spec = (key, nparts, C, nvec, cols, bool(accumulate))
        if not self.active:
            self.rec.append((spec, outs))
            return None
        if self.i >= len(self.layout) or self.layout[self.i] != spec:
            raise RuntimeError("deferred column reductions: the step's producer sequence changed "
                               f"at call {self.i} ({spec[1:]})")
        self.i += 1
        off, rows, *_ = self.regions[key]
        k = self.fill.get(key, 0)
        self.fill[key] = k + nparts
        return self.arena[off + k * C: off + (k + nparts) * C]

    def flush_group(self, g):
        """Reduce the deferred jobs of gradient bucket ``g`` now (its producers are done)."""
        if not self.active or g in self.flushed:
            return
        self.flushed.add(g)
        t = self.tables.get(g)
        if t is not None:
            _lib.call("mx_colreduce_batched", _lib.ptr(t[0]), t[1], t[2], _lib.stream())

    def flush(self):
        """End of backward: reduce every deferred job not reduced yet (one launch per
        group); on the recording step build the layout for the next ones."""
        if self.active:
            if self.i != len(self.layout):
                raise RuntimeError("deferred column reductions: step ended after "
                                   f"{self.i} of {len(self.layout)} producers")
            for g in self.tables:
                self.flush_group(g)
            return
        if not self.rec or torch.cuda.is_current_stream_capturing():
            return
        regions, order, off = {}, [], 0
        for (key, nparts, C, nvec, cols, acc), outs in self.rec:
            if key not in regions:
                regions[key] = [off, 0, C, nvec, cols, outs, acc]
                order.append(key)
            r = regions[key]
            if (r[2], r[3], r[4], r[6]) != (C, nvec, cols, acc) or C % 4:
                return    # (same output with different shapes / unaligned rows: keep immediate mode)
            r[1] += nparts
        # every output pointer belongs to exactly one region, each region to one group
        seen, groups = set(), {}
        for key in order:
            ptrs = [t.data_ptr() for t in regions[key][5] if t is not None]
            if seen.intersection(ptrs) or len(set(ptrs)) != len(ptrs):
                return    # (an output shared by two jobs: a read-modify-write race -> immediate mode)
            seen.update(ptrs)
            gs = {self.group_of(p) for p in ptrs} if self.group_of is not None else {None}
            if len(gs) != 1:
                return    # (one job's outputs in two buckets: cannot be reduced per bucket)
            groups[key] = gs.pop()
        for key in order:           # regions laid out in first-use order
            r = regions[key]
            r[0] = off
            off += r[1] * r[2]
        self.arena = torch.empty(max(off, 1), dtype=torch.float32, device=self.device)
        by_group = {}
        for key in order:
            by_group.setdefault(groups[key], []).append(key)
        self.tables = {}
        for g, keys in by_group.items():
            rows, blk = [], 0
            for key in keys:
                o, nrows, C, nvec, cols, outs, acc = regions[key]
                rows.append([self.arena.data_ptr() + 4 * o, nrows, C, cols] +
                            [(t.data_ptr() if t is not None else 0) for t in outs] + [int(acc), blk])
                blk += (C + 63) // 64
            self.tables[g] = (torch.tensor(rows, dtype=torch.int64).to(self.device), len(rows), blk)
        self.njobs = sum(t[1] for t in self.tables.values())
        self.nblocks = sum(t[2] for t in self.tables.values())
        self.regions = {k: tuple(v) for k, v in regions.items()}
        self.layout = [spec for spec, _ in self.rec]


# ------------------------------------------------------------------ autograd wrappers
class LayerNormFn(torch.autograd.Function):
    """Plain (Rms/Layer)Norm with autograd; parameter grads go to autograd .grad."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps, rms):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        y, mean, rstd = layernorm_fwd(x2, gamma, beta, eps, rms)
        ctx.save_for_backward(x2, mean, rstd, gamma)
        ctx.rms = rms
        ctx.has_beta = beta is not None
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, mean, rstd, gamma = ctx.saved_tensors
        dg = torch.empty_like(gamma)
        db = torch.empty_like(gamma) if ctx.has_beta else None
        dh, _ = norm_bwd(dy.reshape(x2.shape).contiguous(), None, x2, mean, rstd, gamma,
                         rms=ctx.rms, dgamma=dg, dbeta=db)
        return dh.view(ctx.shape), dg, db, None, None


def layer_norm(x, gamma, beta=None, eps=1e-5):
    return LayerNormFn.apply(x, gamma, beta, eps, False)


def rms_norm(x, gamma, eps=1e-6):
    return LayerNormFn.apply(x, gamma, None, eps, True)


class BDANormFn(torch.autograd.Function):
    """y = norm(residual + dropout(x + bias)) with autograd (post-LN transformer blocks,
    e.g. BERT): one fused HIP pass forward, one fused pass backward producing
    d(residual), d(x) (dropout mask regenerated from the seed) and the dgamma/dbeta/dbias
    column sums."""

    @staticmethod
    def forward(ctx, x, bias, residual, gamma, beta, eps, p, seed_t, salt, rms):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        r2 = residual.reshape(-1, shape[-1]).contiguous() if residual is not None else None
        h, y, mean, rstd = bda_norm_fwd(x2, bias, r2, gamma, beta, eps, p, seed_t, salt, rms)
        ctx.save_for_backward(h, mean, rstd, gamma)
        ctx.meta = (p, seed_t, salt, rms, bias is not None, beta is not None, residual is not None, shape)
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        h, mean, rstd, gamma = ctx.saved_tensors
        p, seed_t, salt, rms, has_bias, has_beta, has_res, shape = ctx.meta
        dg = torch.empty_like(gamma)
        db = torch.empty_like(gamma) if has_beta else None
        dbias = torch.empty_like(gamma) if has_bias else None
        dh, dx = norm_bwd(dy.reshape(h.shape).contiguous(), None, h, mean, rstd, gamma, want_dx=True, p=p,
                          seed_t=seed_t, salt=salt, rms=rms, dgamma=dg, dbeta=db, dbias=dbias)
        return (dx.view(shape), dbias, dh.view(shape) if has_res else None, dg, db,
                None, None, None, None, None)


def bda_norm(x, bias, residual, gamma, beta, eps=1e-5, p=0.0, seed_t=None, salt=0, rms=False):
    return BDANormFn.apply(x, bias, residual, gamma, beta, eps, p, seed_t, salt, rms)

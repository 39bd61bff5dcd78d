"""Direct xGMI peer-to-peer collectives (``csrc/comm/xgmi.hip``).

Every rank of a single-node group allocates one registered buffer (+ an uncached flag
block), exports IPC handles, and maps every peer's buffer; the handles travel through
``dist.all_gather_object`` on the group (the c10d store / gloo also work).  A collective
is then ONE kernel that reads from all peers at once -- all 7 xGMI links of an MI355X
carry traffic, where RCCL's ring uses one outbound link per GPU.

    comm = XGMICommunicator(group, device, max_bytes=256 << 20)
    comm.all_reduce_(t)                  # one-shot below ``oneshot_max``, else two-shot
    comm.reduce_scatter(out, inp)        # ZeRO-1 gradient shard
    comm.all_gather(out, inp)            # ZeRO-1 parameter shard
    comm.register("grad", flat_grad)     # collective: map every peer's buffer once
    comm.reduce_scatter_direct(out, "grad", byte_off, nbytes)   # reads peers in place
    comm.all_gather_direct(out, "pshard", byte_off)             # ditto, no copy-in

Validation mode (``MXTRAIN_XGMI_VALIDATE=1``, SURVEY §5.2 race detection): every call
carries a sequence number + signature (op, bytes) that the kernel compares across ranks
after its first barrier (ranks in different collectives -> error word), and the host
checks the result after each call: all-reduce / all-gather outputs must be bit-identical
on every rank (64-bit position-weighted hash, all-gathered), and sum(outputs) must match
sum(inputs) over the group for reductions (fp64, relative 1e-3).  Debug only: it
synchronises after every call.

Selection vs RCCL is explicit: ``MXTRAIN_XGMI=1`` (or ``enable_xgmi()``) routes the
DP reduce-scatter / all-gather and the TP all-reduce through it; ``autotune()`` times
both on the live group and keeps the faster per message-size class.  Barrier waits in
the kernel are bounded; ``check()`` raises if any timed out (a peer never arrived).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops import _lib

OP_ALLREDUCE_1SHOT, OP_ALLREDUCE_2SHOT, OP_REDUCE_SCATTER, OP_ALL_GATHER = 0, 1, 2, 3

_SIGS = {
    "mx_xgmi_handle_size": [],
    "mx_xgmi_flags_bytes": [],
    "mx_xgmi_max_ranks": [],
    "mx_xgmi_alloc": [ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p)],
    "mx_xgmi_free": [ctypes.c_void_p, ctypes.c_void_p],
    "mx_xgmi_get_handle": [ctypes.c_void_p, ctypes.c_void_p],
    "mx_xgmi_open_handle": [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)],
    "mx_xgmi_close_handle": [ctypes.c_void_p],
    "mx_xgmi_error": [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)],
    "mx_xgmi_register": [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64),
                         ctypes.POINTER(ctypes.c_int64)],
    "mx_xgmi_collective": [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_double, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p],
    "mx_xgmi_p2p_ring": [],
    "mx_xgmi_p2p_ctl_bytes": [],
    "mx_xgmi_p2p_alloc": [ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p)],
    "mx_xgmi_p2p_error": [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)],
    "mx_xgmi_p2p": [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                    ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_void_p],
}
OP_RS_DIRECT, OP_AG_DIRECT = 4, 5
ERR_SIG = 0x100


def _hash64(t: torch.Tensor) -> int:
    """Position-weighted 64-bit hash of a tensor's bits (validation mode)."""
    w = t.contiguous().view(-1)
    bits = w.view(torch.int16 if w.element_size() == 2 else torch.int32).to(torch.int64)
    pos = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64).remainder(1 << 20).add(1)
    return int((bits * pos).sum().item())


def _fn(name):
    lib = _lib.lib()
    f = getattr(lib, name)
    f.argtypes = _SIGS[name]
    f.restype = ctypes.c_int
    return f


def _check(err, what):
    if err != 0:
        raise RuntimeError(f"{what} failed with hipError {err}")


class XGMIUnavailable(RuntimeError):
    """Raised on EVERY rank of the group when any rank could not set the communicator up."""


class XGMICommunicator:
    def __init__(self, group, device, max_bytes: int = 256 << 20, oneshot_max: int = 512 << 10,
                 timeout_s: float = 30.0, blocks: int = 0):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device(device)
        assert self.world <= _fn("mx_xgmi_max_ranks")(), "xGMI collectives are single-node (<= 8 ranks)"
        self.max_bytes = (max_bytes + 15) // 16 * 16
        self.oneshot_max = oneshot_max
        self.timeout_s = timeout_s
        self.blocks = blocks
        self._data = ctypes.c_void_p()
        self._flags = ctypes.c_void_p()
        self._opened: List[ctypes.c_void_p] = []
        err = None
        mine = None
        with torch.cuda.device(self.device):
            try:
                _check(_fn("mx_xgmi_alloc")(self.max_bytes, ctypes.byref(self._data),
                                            ctypes.byref(self._flags)), "mx_xgmi_alloc")
                hs = _fn("mx_xgmi_handle_size")()
                hd, hf = ctypes.create_string_buffer(hs), ctypes.create_string_buffer(hs)
                _check(_fn("mx_xgmi_get_handle")(self._data, hd), "hipIpcGetMemHandle(data)")
                _check(_fn("mx_xgmi_get_handle")(self._flags, hf), "hipIpcGetMemHandle(flags)")
                mine = (bytes(hd.raw), bytes(hf.raw))
            except Exception as e:  # keep going: every rank must reach the collectives below
                err = repr(e)
            allh: List = [None] * self.world
            dist.all_gather_object(allh, mine, group=group)
            datas, flags = [], []
            if err is None and all(h is not None for h in allh):
                try:
                    for r, (d, f) in enumerate(allh):
                        if r == self.rank:
                            datas.append(self._data.value)
                            flags.append(self._flags.value)
                            continue
                        pd, pf = ctypes.c_void_p(), ctypes.c_void_p()
                        _check(_fn("mx_xgmi_open_handle")(d, ctypes.byref(pd)),
                               f"hipIpcOpenMemHandle(rank {r})")
                        self._opened.append(pd)
                        _check(_fn("mx_xgmi_open_handle")(f, ctypes.byref(pf)),
                               f"hipIpcOpenMemHandle(rank {r} flags)")
                        self._opened.append(pf)
                        datas.append(pd.value)
                        flags.append(pf.value)
                except Exception as e:
                    err = repr(e)
            elif err is None:
                err = "a peer failed to allocate / export its buffer"
        # every rank learns whether every rank mapped every peer before any kernel runs
        errs: List = [None] * self.world
        dist.all_gather_object(errs, err, group=group)
        bad = [(r, e) for r, e in enumerate(errs) if e is not None]
        if bad:
            self.close()
            raise XGMIUnavailable(f"xGMI communicator setup failed: {bad}")
        self._datas = (ctypes.c_void_p * self.world)(*datas)
        self._flagss = (ctypes.c_void_p * self.world)(*flags)
        self.seq = 0
        self.validate = os.environ.get("MXTRAIN_XGMI_VALIDATE", "0") == "1"
        self.regions: Dict[str, tuple] = {}     # name -> (local ptr, nbytes, [ptr per rank])
        self._mapped: Dict[tuple, int] = {}     # (rank, handle bytes) -> mapped base
        self._region_tensor: Dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ core
    def _launch(self, inp: torch.Tensor, out: torch.Tensor, nbytes: int, op: int, datas=None):
        assert out.is_contiguous() and out.dtype in (torch.bfloat16, torch.float32)
        if inp is not None:
            assert inp.is_contiguous() and out.dtype == inp.dtype
        if op not in (OP_RS_DIRECT, OP_AG_DIRECT) and nbytes > self.max_bytes:
            raise ValueError(f"xGMI message of {nbytes} B (max {self.max_bytes})")
        if nbytes % 16:
            raise ValueError(f"xGMI message of {nbytes} B (must be a multiple of 16)")
        self.seq = (self.seq + 1) & 0xFFFFFFFF
        _check(_fn("mx_xgmi_collective")(datas if datas is not None else self._datas, self._flagss,
                                         self.world, self.rank,
                                         inp.data_ptr() if inp is not None else None, out.data_ptr(), nbytes,
                                         int(out.dtype == torch.bfloat16), op, self.blocks,
                                         self.timeout_s, self.seq, int(self.validate), _lib.stream()),
               "mx_xgmi_collective")

    # ------------------------------------------------------------------ registered buffers
    def register(self, name: str, t: torch.Tensor) -> None:
        """Collective over the group: map every rank's ``t`` (same shape on every rank, e.g.
        the flat gradient buffer) into this process, so direct ops read peers in place.
        ``t`` must stay alive (and not be reallocated) while registered."""
        assert t.is_cuda and t.is_contiguous()
        err, mine = None, None
        try:
            hs = _fn("mx_xgmi_handle_size")()
            h = ctypes.create_string_buffer(hs)
            off, size = ctypes.c_int64(), ctypes.c_int64()
            _check(_fn("mx_xgmi_register")(t.data_ptr(), h, ctypes.byref(off), ctypes.byref(size)),
                   "mx_xgmi_register")
            mine = (bytes(h.raw), off.value, t.numel() * t.element_size())
        except Exception as e:   # every rank must still reach the exchange
            err = repr(e)
        allh: List = [None] * self.world
        dist.all_gather_object(allh, mine, group=self.group)
        ptrs = []
        if err is None:
            try:
                for r, entry in enumerate(allh):
                    if entry is None:
                        raise RuntimeError(f"rank {r} could not export {name}")
                    hb, off, nb = entry
                    if nb != mine[2]:
                        raise RuntimeError(f"{name}: rank {r} registers {nb} B, this rank {mine[2]} B")
                    if r == self.rank:
                        ptrs.append(t.data_ptr())
                        continue
                    key = (r, hb)
                    if key not in self._mapped:
                        pd = ctypes.c_void_p()
                        _check(_fn("mx_xgmi_open_handle")(hb, ctypes.byref(pd)),
                               f"hipIpcOpenMemHandle(rank {r}, {name})")
                        self._opened.append(pd)
                        self._mapped[key] = pd.value
                    ptrs.append(self._mapped[key] + off)
            except Exception as e:
                err = repr(e)
        errs: List = [None] * self.world
        dist.all_gather_object(errs, err, group=self.group)
        bad = [(r, e) for r, e in enumerate(errs) if e is not None]
        if bad:
            raise XGMIUnavailable(f"xGMI register({name}) failed: {bad}")
        self.regions[name] = (t.data_ptr(), t.numel() * t.element_size(), ptrs)
        self._region_tensor[name] = t

    def selftest_direct(self) -> bool:
        """Collective: check the registered-buffer path on this group before real buffers
        use it -- a scratch tensor from the caching allocator (registered at an offset, as
        the flat buffers are) with small-integer data, direct reduce-scatter / all-gather
        vs the staged kernels (exact in bf16), agreed over all ranks."""
        ok = True
        before = set(self._mapped)
        try:
            n = 64 * 1024 * self.world
            big = torch.zeros(n + 4096, dtype=torch.bfloat16, device=self.device)
            buf = big[4096:]
            buf.copy_(torch.arange(n, device=self.device).remainder(7).add(self.rank).to(torch.bfloat16))
            self.register("_selftest", buf)
            a = torch.empty(n // self.world, dtype=torch.bfloat16, device=self.device)
            b = torch.empty_like(a)
            self.reduce_scatter_direct(a, "_selftest", 0, n * 2)
            self.reduce_scatter(b, buf)
            ok = torch.equal(a, b)
            g1 = torch.empty(n, dtype=torch.bfloat16, device=self.device)
            g2 = torch.empty_like(g1)
            self.all_gather_direct(g1, "_selftest", 0)
            self.all_gather(g2, buf[: n // self.world].contiguous())
            ok = ok and torch.equal(g1, g2)
            self.check()
        except Exception:   # noqa: BLE001 -- any failure means: do not use the direct path
            ok = False
        flag = torch.tensor([0.0 if ok else 1.0], device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        self.regions.pop("_selftest", None)
        self._region_tensor.pop("_selftest", None)
        # unmap the scratch segment's peer mappings: its memory returns to the allocator
        torch.cuda.synchronize(self.device)
        for key in set(self._mapped) - before:
            ptr = self._mapped.pop(key)
            for p in self._opened:
                if p.value == ptr:
                    _fn("mx_xgmi_close_handle")(p)
                    p.value = None
        self._opened = [p for p in self._opened if p.value]
        return float(flag.item()) == 0.0

    def has_region(self, name: str, t: Optional[torch.Tensor] = None) -> bool:
        r = self.regions.get(name)
        return r is not None and (t is None or r[0] == t.data_ptr())

    def _region_ptrs(self, name: str, byte_off: int, nbytes: int):
        base, total, ptrs = self.regions[name]
        assert 0 <= byte_off and byte_off + nbytes <= total and byte_off % 16 == 0, (name, byte_off, nbytes)
        return (ctypes.c_void_p * self.world)(*[p + byte_off for p in ptrs])

    def reduce_scatter_direct(self, out: torch.Tensor, name: str, byte_off: int, nbytes: int) -> torch.Tensor:
        """out = shard ``rank`` of the sum over ranks of region[name][byte_off : +nbytes]
        (read in place from every peer's registered buffer)."""
        assert out.numel() * out.element_size() * self.world == nbytes and nbytes % (16 * self.world) == 0
        ptrs = self._region_ptrs(name, byte_off, nbytes)
        if self.validate:
            self._validated("reduce_scatter", out, self._view(name, byte_off, nbytes),
                            lambda: self._launch(None, out, nbytes, OP_RS_DIRECT, ptrs))
            return out
        self._launch(None, out, nbytes, OP_RS_DIRECT, ptrs)
        return out

    def all_gather_direct(self, out: torch.Tensor, name: str, byte_off: int) -> torch.Tensor:
        """out [n * world] = concat over ranks of region[name][byte_off : +n] (every rank's
        shard read in place from its registered buffer)."""
        nb = out.numel() * out.element_size()
        assert nb % (16 * self.world) == 0
        shard_nb = nb // self.world
        ptrs = self._region_ptrs(name, byte_off, shard_nb)
        if self.validate:
            self._validated("all_gather", out, self._view(name, byte_off, shard_nb),
                            lambda: self._launch(None, out, nb, OP_AG_DIRECT, ptrs))
            return out
        self._launch(None, out, nb, OP_AG_DIRECT, ptrs)
        return out

    def _view(self, name, byte_off, nbytes):
        """The local registered bytes [byte_off, +nbytes) as a tensor (validation only)."""
        t = self._region_tensor[name]
        es = t.element_size()
        return t.view(-1)[byte_off // es:(byte_off + nbytes) // es]

    # ------------------------------------------------------------------ validation mode
    def _validated(self, op: str, out: torch.Tensor, inp: torch.Tensor, launch) -> None:
        """Run ``launch`` and check its result across the group (synchronising)."""
        in_sum = float(inp.double().sum()) if op != "all_gather" else 0.0
        seq = self.seq + 1
        launch()
        torch.cuda.synchronize(self.device)
        v = ctypes.c_uint32(0)
        _check(_fn("mx_xgmi_error")(self._flags, ctypes.byref(v)), "mx_xgmi_error")
        errs = []
        if v.value >= ERR_SIG:
            errs.append(f"call signature mismatch with rank {v.value - ERR_SIG} (ranks in different collectives)")
        elif v.value:
            errs.append(f"barrier timeout in phase {v.value - 1}")
        stats = torch.tensor([in_sum, float(out.double().sum())], dtype=torch.float64)
        allstats: List = [None] * self.world
        h = _hash64(out) if op in ("all_reduce", "all_gather") else 0
        dist.all_gather_object(allstats, (stats.tolist(), h, errs), group=self.group)
        if op in ("all_reduce", "all_gather") and len({x[1] for x in allstats}) != 1:
            errs.append("outputs differ across ranks: " + str([x[1] for x in allstats]))
        if op == "all_gather":
            mine = out.view(-1)[self.rank * inp.numel():(self.rank + 1) * inp.numel()]
            if not torch.equal(mine, inp.view(-1)):
                errs.append("own shard not reproduced in the gathered output")
        else:
            tot_in = sum(x[0][0] for x in allstats)
            tot_out = sum(x[0][1] for x in allstats) if op == "reduce_scatter" else allstats[self.rank][0][1]
            if abs(tot_out - tot_in) > 1e-3 * max(1.0, abs(tot_in)) + 1e-2:
                errs.append(f"sum(out)={tot_out:.6g} != sum(in)={tot_in:.6g}")
        others = [(r, x[2]) for r, x in enumerate(allstats) if x[2] and r != self.rank]
        if errs or others:
            raise RuntimeError(f"xGMI validation failed: {op} seq={seq} rank={self.rank}: {errs} peers={others}")

    def supports(self, t: torch.Tensor, shard_multiple: bool = False) -> bool:
        nb = t.numel() * t.element_size()
        ok = t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and nb % 16 == 0
        ok = ok and nb <= self.max_bytes
        if shard_multiple:
            ok = ok and nb % (16 * self.world) == 0
        return ok

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        nb = t.numel() * t.element_size()
        op = OP_ALLREDUCE_1SHOT if nb <= self.oneshot_max else OP_ALLREDUCE_2SHOT
        if self.validate:
            self._validated("all_reduce", t, t.clone(), lambda: self._launch(t, t, nb, op))
            return t
        self._launch(t, t, nb, op)
        return t

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out [n / world] = (sum over ranks of inp [n]) shard ``rank``."""
        nb = inp.numel() * inp.element_size()
        assert out.numel() * self.world == inp.numel() and nb % (16 * self.world) == 0
        if self.validate:
            self._validated("reduce_scatter", out, inp, lambda: self._launch(inp, out, nb, OP_REDUCE_SCATTER))
            return out
        self._launch(inp, out, nb, OP_REDUCE_SCATTER)
        return out

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """out [n * world] = concat over ranks of inp [n]."""
        nb = out.numel() * out.element_size()
        assert inp.numel() * self.world == out.numel() and nb % (16 * self.world) == 0
        if self.validate:
            self._validated("all_gather", out, inp, lambda: self._launch(inp, out, nb, OP_ALL_GATHER))
            return out
        self._launch(inp, out, nb, OP_ALL_GATHER)
        return out

    def check(self):
        """Raise if a barrier in any earlier collective timed out (synchronises)."""
        v = ctypes.c_uint32(0)
        torch.cuda.synchronize(self.device)
        _check(_fn("mx_xgmi_error")(self._flags, ctypes.byref(v)), "mx_xgmi_error")
        if v.value:
            raise RuntimeError(f"xGMI collective barrier timed out on rank {self.rank} "
                               f"(phase {v.value - 1}); a peer never arrived")

    def close(self):
        torch.cuda.synchronize(self.device)
        for p in getattr(self, "_opened", []):
            if p.value:
                _fn("mx_xgmi_close_handle")(p)
        self._opened = []
        self.regions, self._mapped, self._region_tensor = {}, {}, {}
        if getattr(self, "_data", None) is not None and (self._data.value or self._flags.value):
            _fn("mx_xgmi_free")(self._data, self._flags)
        self._data = ctypes.c_void_p()
        self._flags = ctypes.c_void_p()

    # ------------------------------------------------------------------ selection
    # prefer[op] = [(message bytes, xgmi faster?)] measured by autotune(); None = always use
    prefer: Optional[Dict[str, List]] = None
    autotune_ok: Optional[bool] = None

    def use_for(self, op: str, nbytes: int) -> bool:
        if nbytes > self.max_bytes or nbytes % (16 * self.world):
            return False
        if self.prefer is None:
            return True
        table = self.prefer.get(op) or []
        if not table:
            return False
        # nearest measured size class (log scale)
        best = min(table, key=lambda e: abs(math.log2(e[0]) - math.log2(max(nbytes, 16))))
        return bool(best[1])

    def _rccl(self, op, out, inp):
        if op == "all_reduce":
            dist.all_reduce(out, group=self.group)
        elif op == "reduce_scatter":
            dist.reduce_scatter_tensor(out, inp, group=self.group)
        else:
            dist.all_gather_into_tensor(out, inp, group=self.group)

    def _mine(self, op, out, inp):
        if op == "all_reduce":
            self.all_reduce_(out)
        elif op == "reduce_scatter":
            self.reduce_scatter(out, inp)
        else:
            self.all_gather(out, inp)

    def autotune(self, sizes=(1 << 16, 1 << 20, 8 << 20, 64 << 20), iters: int = 8) -> Dict:
        """Check this kernel against RCCL on the live group (integer-valued fp32 data, so
        both must agree exactly) and time both per op and message size.  Timings are
        max-reduced over the ranks so every rank takes the same decision; a mismatch or a
        timed-out barrier on any rank disables the kernel (prefer = {} -> RCCL)."""
        res = {}
        w = self.world
        # the (op, size) grid is the same on every rank, so every collective below -- the
        # RCCL side of each pair and the final max-reductions -- has the same shape everywhere
        keys = [(op, nb) for op in ("all_reduce", "reduce_scatter", "all_gather") for nb in sizes
                if nb <= self.max_bytes and nb % (16 * w) == 0]
        ok = True
        try:
            # fail fast: one small all-reduce with a short barrier bound, checked at once --
            # peers that cannot see each other's flags cost one short timeout, not one 30 s
            # timeout per timed call below
            probe = torch.full((64 * w,), float(self.rank + 1), device=self.device)
            t_keep, self.timeout_s = self.timeout_s, min(self.timeout_s, 5.0)
            try:
                self.all_reduce_(probe)
                self.check()
            finally:
                self.timeout_s = t_keep
            ok = bool((probe == w * (w + 1) / 2).all().item())
        except Exception:
            ok = False
        # the probe's verdict is collective: with one-sided flag visibility one rank can time
        # out while its peer passes, and a rank that skipped the timed loop would leave the
        # peer's RCCL calls below unmatched
        pflag = torch.tensor([1.0 if ok else 0.0], device=self.device)
        dist.all_reduce(pflag, op=dist.ReduceOp.MIN, group=self.group)
        ok = float(pflag.item()) == 1.0
        try:
            for op, nb in (keys if ok else ()):
                n = nb // 4
                big = torch.arange(n, device=self.device, dtype=torch.float32).remainder(13)
                big.add_(self.rank)
                small = big[: n // w].clone()
                inp = big if op == "reduce_scatter" else (small if op == "all_gather" else None)

                def fresh():
                    if op == "all_reduce":
                        return big.clone()
                    return torch.empty(n // w if op == "reduce_scatter" else n, device=self.device)

                a, b = fresh(), fresh()
                self._mine(op, a, inp)
                self._rccl(op, b, inp)
                torch.cuda.synchronize(self.device)
                ok = ok and torch.equal(a, b)
                times = []
                for fn in (self._mine, self._rccl):
                    o = fresh()
                    for _ in range(2):
                        fn(op, o, inp)
                    torch.cuda.synchronize(self.device)
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(iters):
                        fn(op, o, inp)
                    e1.record()
                    torch.cuda.synchronize(self.device)
                    times.append(e0.elapsed_time(e1) / iters)
                res[(op, nb)] = times
            self.check()
        except Exception:
            ok = False
        flag = torch.tensor([0.0 if ok else 1.0], device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        tt = torch.tensor([res.get(k, [0.0, 0.0]) for k in keys] or [[0.0, 0.0]], device=self.device,
                          dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=self.group)
        prefer: Dict[str, List] = {"all_reduce": [], "reduce_scatter": [], "all_gather": []}
        self.autotune_ok = float(flag.item()) == 0.0
        if self.autotune_ok and keys:
            for k, (tx, tr) in zip(keys, tt.tolist()):
                prefer[k[0]].append((k[1], tx < tr))
                res[k] = (tx, tr)
        else:
            prefer = {}
        self.prefer = prefer
        return res


class _P2PHandle:
    """A posted transfer: ``wait()`` makes the current stream wait for it and returns the
    received tensor (None for a send); the send tensor is referenced until then."""
    __slots__ = ("events", "rbuf", "keep")

    def __init__(self, events, rbuf, keep):
        self.events, self.rbuf, self.keep = events, rbuf, keep

    def wait(self):
        cur = torch.cuda.current_stream()
        for e in self.events:
            cur.wait_event(e)
        self.events, self.keep = [], None
        return self.rbuf


class XGMIP2P:
    """Point-to-point channels over xGMI between a rank and its neighbours in ``group``
    (the pipeline group: previous / next stage), for the 1F1B activation / gradient
    transfers (csrc/comm/xgmi.hip p2p_send_kernel / p2p_recv_kernel).  Per peer this rank
    owns a send ring of ``ring`` slots of ``slot_bytes`` and a control block; the peer maps
    both (IPC handles exchanged over the group, collectively).  Sends and receives run on
    two side streams, so a receive waiting for its peer never blocks compute; ``post``
    returns a handle whose ``wait()`` joins the current stream.  Message order per direction
    is the posting order on both sides (the 1F1B schedule is deterministic); the kernels'
    sequence counters live on the device, so a captured schedule replays in step."""

    def __init__(self, group, device, peers, slot_bytes: int, timeout_s: float = 30.0, blocks: int = 32):
        self.group = group
        self.device = torch.device(device)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.slot_bytes = (int(slot_bytes) + 15) // 16 * 16
        self.timeout_s, self.blocks = timeout_s, blocks
        self.peers = sorted({int(p) for p in peers if p is not None and int(p) != self.rank})
        self._ring: Dict[int, ctypes.c_void_p] = {}
        self._ctl: Dict[int, ctypes.c_void_p] = {}
        self._peer_ring: Dict[int, int] = {}
        self._peer_ctl: Dict[int, int] = {}
        self._opened: List[ctypes.c_void_p] = []
        err, mine = None, {}
        with torch.cuda.device(self.device):
            try:
                hs = _fn("mx_xgmi_handle_size")()
                for p in self.peers:
                    r, c = ctypes.c_void_p(), ctypes.c_void_p()
                    _check(_fn("mx_xgmi_p2p_alloc")(self.slot_bytes, ctypes.byref(r), ctypes.byref(c)),
                           "mx_xgmi_p2p_alloc")
                    self._ring[p], self._ctl[p] = r, c
                    hr, hc = ctypes.create_string_buffer(hs), ctypes.create_string_buffer(hs)
                    _check(_fn("mx_xgmi_get_handle")(r, hr), "hipIpcGetMemHandle(p2p ring)")
                    _check(_fn("mx_xgmi_get_handle")(c, hc), "hipIpcGetMemHandle(p2p ctl)")
                    mine[p] = (bytes(hr.raw), bytes(hc.raw))
            except Exception as e:  # every rank must still reach the exchange
                err = repr(e)
            allh: List = [None] * self.world
            dist.all_gather_object(allh, (mine, self.peers), group=group)
            if err is None:
                try:
                    for p in self.peers:
                        theirs, their_peers = allh[p]
                        if self.rank not in their_peers or self.rank not in theirs:
                            raise RuntimeError(f"rank {p} has no channel to rank {self.rank}")
                        hr, hc = theirs[self.rank]
                        pr, pc = ctypes.c_void_p(), ctypes.c_void_p()
                        _check(_fn("mx_xgmi_open_handle")(hr, ctypes.byref(pr)), f"hipIpcOpenMemHandle(p2p ring {p})")
                        self._opened.append(pr)
                        _check(_fn("mx_xgmi_open_handle")(hc, ctypes.byref(pc)), f"hipIpcOpenMemHandle(p2p ctl {p})")
                        self._opened.append(pc)
                        self._peer_ring[p], self._peer_ctl[p] = pr.value, pc.value
                except Exception as e:
                    err = repr(e)
        errs: List = [None] * self.world
        dist.all_gather_object(errs, err, group=group)
        bad = [(r, e) for r, e in enumerate(errs) if e is not None]
        if bad:
            self.close()
            raise XGMIUnavailable(f"xGMI p2p setup failed: {bad}")
        self.s_send = torch.cuda.Stream(device=self.device)
        self.s_recv = torch.cuda.Stream(device=self.device)

    def _launch(self, is_send: bool, peer: int, t: torch.Tensor):
        nb = t.numel() * t.element_size()
        if nb > self.slot_bytes or nb % 16 or not t.is_contiguous():
            raise ValueError(f"xGMI p2p message of {nb} B (slot {self.slot_bytes} B, contiguous, 16-B multiple)")
        ring = self._ring[peer].value if is_send else self._peer_ring[peer]
        _check(_fn("mx_xgmi_p2p")(int(is_send), self._ctl[peer].value, self._peer_ctl[peer], ring,
                                  self.slot_bytes, t.data_ptr(), nb, self.blocks, self.timeout_s, _lib.stream()),
               "mx_xgmi_p2p")

    def post(self, send_t=None, send_to=None, recv_buf=None, recv_from=None) -> _P2PHandle:
        """Post a send of ``send_t`` to group rank ``send_to`` and / or a receive from
        ``recv_from`` into ``recv_buf`` (both allocated on the current stream)."""
        cur = torch.cuda.current_stream(self.device)
        events = []
        keep = None
        if send_t is not None:
            keep = send_t.contiguous()
            self.s_send.wait_stream(cur)
            with torch.cuda.stream(self.s_send):
                self._launch(True, int(send_to), keep)
            events.append(self.s_send.record_event())
        if recv_buf is not None:
            self.s_recv.wait_stream(cur)
            with torch.cuda.stream(self.s_recv):
                self._launch(False, int(recv_from), recv_buf)
            events.append(self.s_recv.record_event())
        return _P2PHandle(events, recv_buf, keep)

    def selftest(self, timeout_s: float = 5.0) -> bool:
        """Round-trip a known tensor with every peer (both directions at once: sends and
        receives run on their own streams) under a short wait bound and compare; the verdict
        is agreed over the group (MIN), so every rank keeps or drops the channels together.
        Collective: call on every rank of the group, before any real traffic."""
        ok = True
        t_keep, self.timeout_s = self.timeout_s, min(self.timeout_s, timeout_s)
        try:
            n = min(self.slot_bytes // 4, 4096) // 4 * 4
            hs = []
            for p in self.peers:
                src = torch.arange(n, device=self.device, dtype=torch.float32).add_(1000.0 * self.rank + 7 * p)
                dst = torch.full((n,), -1.0, device=self.device)
                hs.append((p, self.post(src, p, dst, p), dst))
            for p, h, dst in hs:
                got = h.wait()
                exp = torch.arange(n, device=self.device, dtype=torch.float32).add_(1000.0 * p + 7 * self.rank)
                ok = ok and bool(torch.equal(got, exp))
            self.check()
        except Exception:
            ok = False
        finally:
            self.timeout_s = t_keep
        flag = torch.tensor([1.0 if ok else 0.0], device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return float(flag.item()) == 1.0

    def check(self):
        """Raise if a send / receive wait timed out on this rank (synchronises)."""
        torch.cuda.synchronize(self.device)
        for p, c in self._ctl.items():
            v = ctypes.c_uint32(0)
            _check(_fn("mx_xgmi_p2p_error")(c, ctypes.byref(v)), "mx_xgmi_p2p_error")
            if v.value:
                raise RuntimeError(f"xGMI p2p {'send' if v.value == 1 else 'receive'} with rank {p} timed out "
                                   f"on rank {self.rank}")

    def close(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize(self.device)
        for p in self._opened:
            if p.value:
                _fn("mx_xgmi_close_handle")(p)
        self._opened = []
        for p in list(self._ring):
            _fn("mx_xgmi_free")(self._ring[p], self._ctl[p])
        self._ring, self._ctl = {}, {}


_P2PS: Dict[tuple, Optional[XGMIP2P]] = {}


def get_p2p(group, device, peers, slot_bytes: int) -> Optional[XGMIP2P]:
    """The pipeline group's xGMI p2p channels when ``MXTRAIN_XGMI`` is 1 / auto (GPU, one
    node), else None (RCCL batch_isend_irecv).  Collective over ``group`` on first use."""
    if not enabled() or group is None or not torch.cuda.is_available():
        return None
    key = (id(group), tuple(sorted(p for p in peers if p is not None)), int(slot_bytes))
    if key in _P2PS:
        return _P2PS[key]
    if torch.cuda.is_current_stream_capturing():
        return None
    c = None
    if _single_node(group):
        try:
            c = XGMIP2P(group, device, peers, slot_bytes,
                        timeout_s=float(os.environ.get("MXTRAIN_XGMI_TIMEOUT_S", "30")))
        except XGMIUnavailable as e:
            if dist.get_rank(group) == 0:
                print(f"[mxtrain] {e}; pipeline p2p uses RCCL", flush=True)
        # validated once against known data (agreed on every rank): a channel whose waits
        # time out would otherwise leave the receive buffer unwritten and train on garbage
        if c is not None and not c.selftest():
            if dist.get_rank(group) == 0:
                print("[mxtrain] xGMI p2p self-test failed; pipeline p2p uses RCCL", flush=True)
            c.close()
            c = None
    _P2PS[key] = c
    return c


_NODE: Dict[int, bool] = {}


def _single_node(group) -> bool:
    """Whether every rank of ``group`` runs on this host (collective on first use): the
    xGMI kernels map peer memory through IPC handles, which exist within one node only."""
    key = id(group)
    if key not in _NODE:
        import socket
        names: List = [None] * dist.get_world_size(group)
        dist.all_gather_object(names, socket.gethostname(), group=group)
        _NODE[key] = len(set(names)) == 1
    return _NODE[key]


_COMMS: Dict[int, Optional[XGMICommunicator]] = {}


def mode() -> str:
    """MXTRAIN_XGMI: 0 = RCCL only (default), 1 = xGMI kernels for every supported
    message, auto = check + time both on the live group and keep the faster per size."""
    return os.environ.get("MXTRAIN_XGMI", "0")


def enabled() -> bool:
    return mode() in ("1", "auto")


def direct_enabled() -> bool:
    """MXTRAIN_XGMI_DIRECT (default 1): ZeRO-1 buckets use the registered-buffer kernels."""
    return os.environ.get("MXTRAIN_XGMI_DIRECT", "1") == "1"


def enable_xgmi(on="1"):
    os.environ["MXTRAIN_XGMI"] = {True: "1", False: "0"}.get(on, on)


def get_comm(group, device) -> Optional[XGMICommunicator]:
    """The group's communicator when xGMI collectives are enabled and usable (GPU, one
    node, <= 8 ranks), else None (callers use RCCL)."""
    if not enabled() or group is None or not torch.cuda.is_available():
        return None
    if dist.get_world_size(group) == 1:
        return None
    key = id(group)
    if key in _COMMS:
        return _COMMS[key]
    if not _single_node(group):
        _COMMS[key] = None
        return None
    max_mb = int(os.environ.get("MXTRAIN_XGMI_MAX_MB", "256"))
    try:
        c = XGMICommunicator(group, device, max_bytes=max_mb << 20,
                             timeout_s=float(os.environ.get("MXTRAIN_XGMI_TIMEOUT_S", "30")))
    except XGMIUnavailable as e:   # agreed on every rank -> RCCL everywhere
        if dist.get_rank(group) == 0:
            print(f"[mxtrain] {e}; using RCCL", flush=True)
        c = None
    if c is not None and mode() == "auto":
        c.autotune()
        if dist.get_rank(group) == 0:
            print(f"[mxtrain] xGMI autotune (world {c.world}): ok={c.autotune_ok} prefer={c.prefer}",
                  flush=True)
    _COMMS[key] = c
    return c


def route(group, t: torch.Tensor, op: str, nbytes: int) -> Optional[XGMICommunicator]:
    """Communicator to use for this call, or None for RCCL.  Never builds a communicator
    while a hipGraph is being captured (allocation + handle exchange are not capturable)."""
    if not enabled() or group is None or not t.is_cuda:
        return None
    if id(group) not in _COMMS and torch.cuda.is_current_stream_capturing():
        return None   # (build it eagerly first: e.g. warmup steps before the graph capture)
    c = get_comm(group, t.device)
    if c is None or not c.use_for(op, nbytes):
        return None
    return c


def destroy_all():
    for c in list(_COMMS.values()) + list(_P2PS.values()):
        if c is not None:
            c.close()
    _COMMS.clear()
    _P2PS.clear()
    _NODE.clear()

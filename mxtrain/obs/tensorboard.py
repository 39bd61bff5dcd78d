"""TensorBoard event files without TensorFlow (C10/C11 in-pod TensorBoard,
C44 Kubeflow Tensorboards ``Tensorboard.spec.logspath``).

``SummaryWriter(logdir).add_scalar(tag, value, step)`` writes
``events.out.tfevents.<time>.<host>`` in the standard TFRecord framing (length, masked
CRC-32C of the length, payload, masked CRC-32C of the payload) with hand-encoded
``tensorflow.Event`` / ``Summary`` protobuf messages, so any TensorBoard (or the
dashboard in ``mxtrain.mlplatform.dashboard``) can read the runs.  CRC-32C comes from the
native runtime library (``csrc/runtime/crc32c.cpp``, SSE4.2 ``crc32``); a pure-Python
table is the fallback.  ``read_scalars(logdir)`` parses the same files back.

Megatron's ``--tensorboard-dir`` and tensorpack's ``train_log`` use it.
"""
from __future__ import annotations

import ctypes
import glob
import os
import socket
import struct
import time
from typing import Dict, List, Tuple

# ---------------------------------------------------------------------------- crc32c
_PY_TABLE = None
_NATIVE = None


def _native():
    global _NATIVE
    if _NATIVE is None:
        try:
            from ..runtime import native
            L = native.lib()
            L.mx_masked_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
            L.mx_masked_crc32c.restype = ctypes.c_uint32
            _NATIVE = L
        except Exception:
            _NATIVE = False
    return _NATIVE


def _py_crc32c(data: bytes) -> int:
    global _PY_TABLE
    if _PY_TABLE is None:
        t = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
            t.append(c)
        _PY_TABLE = t
    c = 0xFFFFFFFF
    for b in data:
        c = (c >> 8) ^ _PY_TABLE[(c ^ b) & 0xFF]
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    L = _native()
    if L:
        return int(L.mx_masked_crc32c(data, len(data)))
    c = _py_crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------------------- protobuf
def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_event(wall_time: float, step: int = 0, file_version: str = None,
                 scalars: Dict[str, float] = None) -> bytes:
    msg = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        msg += _len_field(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, v in scalars.items():
            val = _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v))
            summ += _len_field(1, val)
        msg += _len_field(5, summ)
    return msg


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = n = 0
    while True:
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        if not b & 0x80:
            return n, i
        shift += 7


def _fields(buf: bytes):
    i = 0
    while i < len(buf):
        k, i = _read_varint(buf, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(buf, i)
        elif w == 1:
            v = buf[i:i + 8]
            i += 8
        elif w == 5:
            v = buf[i:i + 4]
            i += 4
        elif w == 2:
            ln, i = _read_varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        else:
            raise ValueError(f"unsupported wire type {w}")
        yield f, w, v


def decode_event(buf: bytes) -> dict:
    ev = {"wall_time": 0.0, "step": 0, "scalars": {}}
    for f, w, v in _fields(buf):
        if f == 1 and w == 1:
            ev["wall_time"] = struct.unpack("<d", v)[0]
        elif f == 2 and w == 0:
            ev["step"] = v
        elif f == 3 and w == 2:
            ev["file_version"] = v.decode()
        elif f == 5 and w == 2:
            for f2, _, val in _fields(v):
                if f2 != 1:
                    continue
                tag, x = None, None
                for f3, w3, v3 in _fields(val):
                    if f3 == 1:
                        tag = v3.decode()
                    elif f3 == 2 and w3 == 5:
                        x = struct.unpack("<f", v3)[0]
                if tag is not None and x is not None:
                    ev["scalars"][tag] = x
    return ev


# ---------------------------------------------------------------------------- records
def _record(payload: bytes) -> bytes:
    hdr = struct.pack("<Q", len(payload))
    return hdr + struct.pack("<I", masked_crc32c(hdr)) + payload + struct.pack("<I", masked_crc32c(payload))


def read_records(path: str, verify: bool = True):
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i + 12 <= len(data):
        hdr = data[i:i + 8]
        (n,) = struct.unpack("<Q", hdr)
        (hc,) = struct.unpack("<I", data[i + 8:i + 12])
        if verify and hc != masked_crc32c(hdr):
            raise ValueError(f"{path}: corrupt record header at {i}")
        if i + 12 + n + 4 > len(data):
            break  # partially written tail
        payload = data[i + 12:i + 12 + n]
        (pc,) = struct.unpack("<I", data[i + 12 + n:i + 16 + n])
        if verify and pc != masked_crc32c(payload):
            raise ValueError(f"{path}: corrupt record payload at {i}")
        yield payload
        i += 16 + n


class SummaryWriter:
    """Minimal tensorboardX/torch.utils.tensorboard-compatible scalar writer."""

    def __init__(self, logdir: str, flush_secs: float = 10.0, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        fn = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}{filename_suffix}"
        self.path = os.path.join(logdir, fn)
        self._f = open(self.path, "ab")
        self._f.write(_record(encode_event(time.time(), 0, file_version="brain.Event:2")))
        self._last_flush = time.time()
        self.flush_secs = flush_secs

    def add_scalar(self, tag: str, value: float, global_step: int = 0, walltime: float = None):
        self.add_scalars_flat({tag: value}, global_step, walltime)

    def add_scalars_flat(self, values: Dict[str, float], global_step: int = 0, walltime: float = None):
        self._f.write(_record(encode_event(walltime or time.time(), global_step, scalars=values)))
        if time.time() - self._last_flush > self.flush_secs:
            self.flush()

    def flush(self):
        self._f.flush()
        self._last_flush = time.time()

    def close(self):
        if self._f:
            self._f.flush()
            self._f.close()
            self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def event_files(logdir: str) -> List[str]:
    return sorted(glob.glob(os.path.join(logdir, "**", "events.out.tfevents.*"), recursive=True))


def read_scalars(logdir: str) -> Dict[str, List[Tuple[int, float, float]]]:
    """{run/tag: [(step, wall_time, value), ...]} over every event file under logdir
    (run = event file's directory relative to logdir)."""
    out: Dict[str, List[Tuple[int, float, float]]] = {}
    for p in event_files(logdir):
        run = os.path.relpath(os.path.dirname(p), logdir)
        for payload in read_records(p):
            ev = decode_event(payload)
            for tag, v in ev["scalars"].items():
                key = tag if run == "." else f"{run}/{tag}"
                out.setdefault(key, []).append((ev["step"], ev["wall_time"], v))
    for v in out.values():
        v.sort()
    return out

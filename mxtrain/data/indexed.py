"""Memory-mapped indexed token dataset, byte-compatible with the Megatron "mmap"
format that `tools/preprocess_data.py --dataset-impl mmap` writes and
`pretrain_gpt.py --data-impl mmap --data-path <prefix>` reads (SURVEY §2.11, §3.5:
`gpt2_text_document.{bin,idx}`).

``<prefix>.bin``  the token ids of every sequence, back to back, in ``dtype``.
``<prefix>.idx``  header + three arrays::

    9s  magic  b"MMIDIDX\\x00\\x00"
    <Q  version (1)
    <B  dtype code  (1 u8, 2 i8, 3 i16, 4 i32, 5 i64, 6 f64, 7 f64, 8 u16)
    <Q  number of sequences  N
    <Q  number of document boundaries  M
    int32[N]  sequence lengths (tokens)
    int64[N]  byte offset of each sequence in .bin
    int64[M]  document index: sequence index where each document starts (+ final N)

Reading maps both files (no copy); a sequence is a zero-copy numpy view.
"""
from __future__ import annotations

import os
import struct
from typing import Iterable, List, Optional

import numpy as np

MAGIC = b"MMIDIDX\x00\x00"
DTYPES = {1: np.uint8, 2: np.int8, 3: np.int16, 4: np.int32, 5: np.int64, 6: np.float64,
          7: np.float64, 8: np.uint16}
CODES = {np.dtype(np.uint8): 1, np.dtype(np.int8): 2, np.dtype(np.int16): 3, np.dtype(np.int32): 4,
         np.dtype(np.int64): 5, np.dtype(np.float64): 7, np.dtype(np.uint16): 8}


def best_fitting_dtype(vocab_size: Optional[int]):
    return np.uint16 if vocab_size is not None and vocab_size < 65500 else np.int32


def data_file_path(prefix: str) -> str:
    return prefix + ".bin"


def index_file_path(prefix: str) -> str:
    return prefix + ".idx"


def exists(prefix: str) -> bool:
    return os.path.exists(data_file_path(prefix)) and os.path.exists(index_file_path(prefix))


class IndexedDatasetBuilder:
    def __init__(self, bin_path: str, dtype=np.uint16):
        self.dtype = np.dtype(dtype)
        self._f = open(bin_path, "wb")
        self.sizes: List[int] = []
        self.doc_idx: List[int] = [0]

    def add_item(self, tokens: Iterable[int]):
        arr = np.asarray(tokens, dtype=self.dtype)
        self._f.write(arr.tobytes(order="C"))
        self.sizes.append(int(arr.size))

    def end_document(self):
        self.doc_idx.append(len(self.sizes))

    def merge_file_(self, prefix: str):
        other = MMapIndexedDataset(prefix)
        assert other.dtype == self.dtype
        base = len(self.sizes)
        self.sizes.extend(int(s) for s in other.sizes)
        self.doc_idx.extend(int(d) + base for d in other.doc_idx[1:])
        with open(data_file_path(prefix), "rb") as f:
            while True:
                chunk = f.read(1 << 24)
                if not chunk:
                    break
                self._f.write(chunk)

    def finalize(self, idx_path: str):
        self._f.close()
        write_index(idx_path, self.dtype, self.sizes, self.doc_idx)


def write_index(idx_path: str, dtype, sizes, doc_idx):
    dtype = np.dtype(dtype)
    sizes = np.asarray(sizes, dtype=np.int32)
    pointers = np.zeros(len(sizes), dtype=np.int64)
    if len(sizes) > 1:
        np.cumsum(sizes[:-1].astype(np.int64) * dtype.itemsize, out=pointers[1:])
    doc_idx = np.asarray(doc_idx, dtype=np.int64)
    with open(idx_path, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<Q", 1))
        f.write(struct.pack("<B", CODES[dtype]))
        f.write(struct.pack("<Q", len(sizes)))
        f.write(struct.pack("<Q", len(doc_idx)))
        f.write(sizes.tobytes(order="C"))
        f.write(pointers.tobytes(order="C"))
        f.write(doc_idx.tobytes(order="C"))


class MMapIndexedDataset:
    def __init__(self, prefix: str):
        self.prefix = prefix
        with open(index_file_path(prefix), "rb") as f:
            magic = f.read(9)
            if magic != MAGIC:
                raise ValueError(f"{prefix}.idx: not an mmap indexed dataset (bad magic)")
            (version,) = struct.unpack("<Q", f.read(8))
            if version != 1:
                raise ValueError(f"{prefix}.idx: unsupported version {version}")
            (code,) = struct.unpack("<B", f.read(1))
            self.dtype = np.dtype(DTYPES[code])
            (n,) = struct.unpack("<Q", f.read(8))
            (m,) = struct.unpack("<Q", f.read(8))
            offset = f.tell()
        self._idx = np.memmap(index_file_path(prefix), mode="r", order="C")
        self.sizes = np.frombuffer(self._idx, dtype=np.int32, count=n, offset=offset)
        self.pointers = np.frombuffer(self._idx, dtype=np.int64, count=n, offset=offset + self.sizes.nbytes)
        self.doc_idx = np.frombuffer(self._idx, dtype=np.int64, count=m,
                                     offset=offset + self.sizes.nbytes + self.pointers.nbytes)
        nbytes = os.path.getsize(data_file_path(prefix))
        self._bin = np.memmap(data_file_path(prefix), mode="r", order="C") if nbytes else np.zeros(0, np.uint8)

    def __len__(self):
        return len(self.sizes)

    def __getitem__(self, i: int) -> np.ndarray:
        return np.frombuffer(self._bin, dtype=self.dtype, count=int(self.sizes[i]), offset=int(self.pointers[i]))

    def get(self, i: int, offset: int = 0, length: Optional[int] = None) -> np.ndarray:
        if length is None:
            length = int(self.sizes[i]) - offset
        ptr = int(self.pointers[i]) + offset * self.dtype.itemsize
        return np.frombuffer(self._bin, dtype=self.dtype, count=length, offset=ptr)

    @property
    def num_documents(self):
        return len(self.doc_idx) - 1

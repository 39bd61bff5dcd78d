"""GPT pre-training datasets (Megatron `--data-path ... --data-impl mmap --split 949,50,1
--data-cache-path ...` semantics; mock data for synthetic runs).

A split is a contiguous range of documents.  Per split the sample stream is built the
Megatron way:

* ``doc_idx``     the split's documents repeated for enough epochs, each epoch shuffled;
* ``sample_idx``  for sample s, (position in doc_idx, token offset) where it starts --
                  built natively (csrc/runtime/dataset_helpers.cpp);
* ``shuffle_idx`` a permutation of the samples.

All three are cached as .npy under ``--data-cache-path`` (keyed by a hash of the
description), so every rank and every restart reuses them.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..runtime import native
from .indexed import MMapIndexedDataset


def parse_split(split: str) -> List[float]:
    parts = [float(x) for x in split.replace("/", ",").split(",") if x.strip()]
    while len(parts) < 3:
        parts.append(0.0)
    s = sum(parts)
    return [p / s for p in parts[:3]]


def split_boundaries(split: str, ndocs: int) -> List[int]:
    fr = parse_split(split)
    idx = [0]
    for f in fr:
        idx.append(idx[-1] + int(round(f * float(ndocs))))
    diff = idx[-1] - ndocs
    for i in range(1, len(idx)):
        idx[i] -= diff
    return idx


class GPTDataset(torch.utils.data.Dataset):
    def __init__(self, name: str, indexed: MMapIndexedDataset, documents: np.ndarray, num_samples: int,
                 seq_length: int, seed: int, cache_dir: Optional[str] = None):
        self.name, self.ds, self.seq_length = name, indexed, seq_length
        documents = np.asarray(documents, dtype=np.int32)
        assert documents.size > 0, f"{name} split has no documents"
        desc = {"class": "GPTDataset", "prefix": os.path.abspath(indexed.prefix), "split": name,
                "docs": [int(documents[0]), int(documents[-1]), int(documents.size)],
                "num_samples": int(num_samples), "seq_length": seq_length, "seed": seed}
        key = hashlib.md5(json.dumps(desc, sort_keys=True).encode()).hexdigest()
        cache_dir = cache_dir or os.path.join(os.path.dirname(os.path.abspath(indexed.prefix)), "cache")
        base = os.path.join(cache_dir, f"{key}-{name}")
        files = [base + s for s in ("-doc_idx.npy", "-sample_idx.npy", "-shuffle_idx.npy")]
        if all(os.path.exists(f) for f in files):
            self.doc_idx, self.sample_idx, self.shuffle_idx = (np.load(f, mmap_mode="r") for f in files)
            return
        sizes = np.asarray(indexed.sizes, dtype=np.int32)
        tokens_per_epoch = int(sizes[documents].astype(np.int64).sum())
        assert tokens_per_epoch > seq_length, f"{name}: not enough tokens for one sample"
        epochs = 1
        while native.sample_count(epochs, tokens_per_epoch, seq_length) < num_samples:
            epochs += 1
        rng = np.random.RandomState(seed)
        doc_idx = np.concatenate([rng.permutation(documents) for _ in range(epochs)]).astype(np.int32)
        total = native.sample_count(epochs, tokens_per_epoch, seq_length)
        sample_idx = native.build_sample_idx(sizes, doc_idx, seq_length, total)
        shuffle_idx = rng.permutation(total).astype(np.int64)
        os.makedirs(cache_dir, exist_ok=True)
        for f, a in zip(files, (doc_idx, sample_idx, shuffle_idx)):
            tmp = f + f".{os.getpid()}.tmp.npy"
            np.save(tmp, a)
            os.replace(tmp, f)
        with open(base + "-desc.json", "w") as fh:
            json.dump(desc, fh, indent=1)
        self.doc_idx, self.sample_idx, self.shuffle_idx = doc_idx, sample_idx, shuffle_idx

    def __len__(self):
        return len(self.shuffle_idx)

    def tokens(self, idx: int) -> np.ndarray:
        j = int(self.shuffle_idx[idx % len(self.shuffle_idx)])
        d0, o0 = (int(x) for x in self.sample_idx[j])
        d1, o1 = (int(x) for x in self.sample_idx[j + 1])
        if d0 == d1:
            return np.asarray(self.ds.get(int(self.doc_idx[d0]), o0, o1 - o0 + 1), dtype=np.int64)
        parts = [self.ds.get(int(self.doc_idx[d0]), o0)]
        for d in range(d0 + 1, d1):
            parts.append(self.ds.get(int(self.doc_idx[d])))
        parts.append(self.ds.get(int(self.doc_idx[d1]), 0, o1 + 1))
        return np.concatenate(parts).astype(np.int64)

    def __getitem__(self, idx):
        return {"text": torch.from_numpy(self.tokens(idx))}


class MockGPTDataset(torch.utils.data.Dataset):
    """Deterministic synthetic token samples (`--mock-data`; the box has no corpus)."""

    def __init__(self, num_samples: int, seq_length: int, vocab_size: int, seed: int):
        self.n, self.s, self.v, self.seed = num_samples, seq_length, vocab_size, seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        return {"text": torch.randint(0, self.v, (self.s + 1,), generator=g, dtype=torch.int64)}


def build_train_valid_test(data_prefix: Optional[str], split: str, num_samples: Sequence[int], seq_length: int,
                           seed: int, cache_dir: Optional[str] = None, vocab_size: int = 50257,
                           mock: bool = False):
    if mock or not data_prefix:
        return [MockGPTDataset(max(n, 1), seq_length, vocab_size, seed + i) if n > 0 else None
                for i, n in enumerate(num_samples)]
    ds = MMapIndexedDataset(data_prefix)
    b = split_boundaries(split, len(ds.sizes))
    out = []
    for i, (name, n) in enumerate(zip(("train", "valid", "test"), num_samples)):
        if n <= 0 or b[i + 1] <= b[i]:
            out.append(None)
            continue
        out.append(GPTDataset(name, ds, np.arange(b[i], b[i + 1], dtype=np.int32), n, seq_length, seed, cache_dir))
    return out


class DistributedSampleLoader:
    """Megatron's pretraining sampler: consecutive global batches, each DP rank takes its
    micro-batches of every global batch; resumable from consumed_samples."""

    def __init__(self, dataset, micro_batch: int, global_batch: int, dp_rank: int, dp: int,
                 consumed_samples: int = 0):
        self.ds, self.mb, self.gb, self.r, self.dp = dataset, micro_batch, global_batch, dp_rank, dp
        self.consumed = consumed_samples
        assert global_batch % (micro_batch * dp) == 0
        self.num_micro = global_batch // (micro_batch * dp)

    def next_batch(self):
        """[num_micro, micro_batch, seq+1] int64 for this rank."""
        base = self.consumed
        per_rank = self.mb * self.num_micro
        rows = []
        for k in range(per_rank):
            # rank r owns a contiguous block of the global batch, like Megatron's sampler
            idx = base + self.r * per_rank + k
            rows.append(self.ds[idx % len(self.ds)]["text"])
        self.consumed += self.gb
        x = torch.stack(rows).view(self.num_micro, self.mb, -1)
        return x

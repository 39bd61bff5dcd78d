"""JSON-lines corpus -> Megatron mmap indexed dataset, command-line compatible with
Megatron-DeepSpeed's `tools/preprocess_data.py` as the reference's wikicorpus example
runs it (examples/megatron-deepspeed/gpt2_345m/wikicorpus.yaml:31-42):

    python3 tools/preprocess_data.py --input $DATA_ROOT/train.json \\
        --output-prefix $DATA_ROOT/gpt2 --vocab-file gpt2-vocab.json --dataset-impl mmap \\
        --tokenizer-type GPT2BPETokenizer --merge-file gpt2-merges.txt --append-eod --workers 4

Output: ``<output-prefix>_<json-key>_document.{bin,idx}`` (e.g. gpt2_text_document).
Workers tokenise disjoint line ranges in parallel (``--workers`` processes, each using the
Rust BPE core on batches); partial outputs are merged in input order.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))))))

from mxtrain.data.indexed import (IndexedDatasetBuilder, best_fitting_dtype, data_file_path,  # noqa: E402
                                  index_file_path)
from mxtrain.data.tokenizer import build_tokenizer  # noqa: E402


def get_args(argv=None):
    p = argparse.ArgumentParser(allow_abbrev=False)
    g = p.add_argument_group("input data")
    g.add_argument("--input", required=True)
    g.add_argument("--json-keys", nargs="+", default=["text"])
    g.add_argument("--split-sentences", action="store_true")
    g.add_argument("--keep-newlines", action="store_true")
    g = p.add_argument_group("tokenizer")
    g.add_argument("--tokenizer-type", default="GPT2BPETokenizer")
    g.add_argument("--vocab-file", default=None)
    g.add_argument("--merge-file", default=None)
    g.add_argument("--vocab-size", type=int, default=None)
    g.add_argument("--append-eod", action="store_true")
    g.add_argument("--lang", default="english")
    g = p.add_argument_group("output data")
    g.add_argument("--output-prefix", required=True)
    g.add_argument("--dataset-impl", default="mmap", choices=["lazy", "cached", "mmap"])
    g = p.add_argument_group("runtime")
    g.add_argument("--workers", type=int, default=1)
    g.add_argument("--partitions", type=int, default=1)
    g.add_argument("--chunk-size", type=int, default=256)
    g.add_argument("--log-interval", type=int, default=10000)
    a = p.parse_args(argv)
    if a.dataset_impl != "mmap":
        print(f"[mxtrain] --dataset-impl {a.dataset_impl}: writing mmap (the only on-disk format used)")
    return a


_TOK = None


def _init(args):
    global _TOK
    _TOK = build_tokenizer(args.tokenizer_type, args.vocab_file, args.merge_file, args.vocab_size)


def _split_sentences(text):
    import re
    return [s for s in re.split(r"(?<=[.!?])\s+", text) if s]


def _work(job):
    """Tokenise lines [start, end) of the input into <tmp>.{bin,idx}."""
    args, start, end, tmp_prefix = job
    _init(args)
    dtype = best_fitting_dtype(_TOK.vocab_size)
    builders = {k: IndexedDatasetBuilder(data_file_path(f"{tmp_prefix}_{k}"), dtype) for k in args.json_keys}
    ndocs = 0
    ntok = 0
    with open(args.input, encoding="utf-8") as f:
        batch = []
        for li, line in enumerate(f):
            if li < start:
                continue
            if li >= end:
                break
            if not line.strip():
                continue
            batch.append(json.loads(line))
            if len(batch) >= args.chunk_size:
                ntok += _flush(args, batch, builders)
                ndocs += len(batch)
                batch = []
        if batch:
            ntok += _flush(args, batch, builders)
            ndocs += len(batch)
    for k, b in builders.items():
        b.finalize(index_file_path(f"{tmp_prefix}_{k}"))
    return ndocs, ntok


def _flush(args, batch, builders):
    ntok = 0
    for k, b in builders.items():
        texts = [str(doc.get(k, "")) for doc in batch]
        if args.split_sentences:
            for t in texts:
                sents = _split_sentences(t)
                ids = _TOK.tokenize_batch(sents) if sents else []
                for j, s in enumerate(ids):
                    if args.append_eod and j == len(ids) - 1:
                        s = s + [_TOK.eod]
                    if s:
                        b.add_item(s)
                        ntok += len(s)
                b.end_document()
        else:
            for s in _TOK.tokenize_batch(texts):
                if args.append_eod:
                    s = s + [_TOK.eod]
                if s:
                    b.add_item(s)
                    ntok += len(s)
                b.end_document()
    return ntok


def main(argv=None):
    args = get_args(argv)
    t0 = time.time()
    with open(args.input, encoding="utf-8") as f:
        nlines = sum(1 for _ in f)
    w = max(1, min(args.workers, nlines))
    per = (nlines + w - 1) // w
    tmp = [f"{args.output_prefix}.part{i}" for i in range(w)]
    jobs = [(args, i * per, min(nlines, (i + 1) * per), tmp[i]) for i in range(w)]
    print(f"Opening {args.input}: {nlines} documents, {w} workers", flush=True)
    if w == 1:
        results = [_work(jobs[0])]
    else:
        with mp.get_context("spawn").Pool(w) as pool:
            results = pool.map(_work, jobs)
    _init(args)
    dtype = best_fitting_dtype(_TOK.vocab_size)
    for k in args.json_keys:
        level = "sentence" if args.split_sentences else "document"
        out = f"{args.output_prefix}_{k}_{level}"
        b = IndexedDatasetBuilder(data_file_path(out), dtype)
        for t in tmp:
            b.merge_file_(f"{t}_{k}")
        b.finalize(index_file_path(out))
        for t in tmp:
            for suf in (".bin", ".idx"):
                os.unlink(f"{t}_{k}{suf}")
        print(f"Output prefix: {out}", flush=True)
    ndocs = sum(r[0] for r in results)
    ntok = sum(r[1] for r in results)
    dt = time.time() - t0
    print(f"Processed {ndocs} documents, {ntok} tokens in {dt:.1f}s ({ndocs / max(dt, 1e-9):.1f} docs/s, "
          f"{ntok / max(dt, 1e-9) / 1e6:.2f} M tokens/s)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

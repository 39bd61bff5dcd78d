"""GPT-2 byte-level BPE tokenizer (Megatron `--tokenizer-type GPT2BPETokenizer
--vocab-file gpt2-vocab.json --merge-file gpt2-merges.txt`) on the HF `tokenizers`
Rust core, plus an offline replacement for Megatron's `dataset/download_vocab.sh`.

The node cannot download the real GPT-2 vocabulary, so ``make_gpt2_vocab`` trains a
byte-level BPE on a local corpus (or a synthetic one) and lays it out exactly like
GPT-2's files: 50257 entries, ``<|endoftext|>`` = 50256, merges in rank order.  The
vocabulary *size* is what determines the model (padded to 50304 for TP=1), so GPT-2
345M shapes are unchanged.
"""
from __future__ import annotations

import json
import os
from typing import Iterable, List, Optional

GPT2_VOCAB_SIZE = 50257
EOD = "<|endoftext|>"


def make_gpt2_vocab(vocab_file: str, merge_file: str, corpus: Optional[Iterable[str]] = None,
                    vocab_size: int = GPT2_VOCAB_SIZE, seed: int = 0):
    from tokenizers import ByteLevelBPETokenizer
    if corpus is None:
        from .text_synth import TextGen
        g = TextGen(seed)
        corpus = [g.document() for _ in range(2000)]
    tok = ByteLevelBPETokenizer()
    tok.train_from_iterator(corpus, vocab_size=vocab_size - 1, min_frequency=2, special_tokens=[])
    tmp = os.path.dirname(os.path.abspath(vocab_file)) or "."
    os.makedirs(tmp, exist_ok=True)
    files = tok.save_model(tmp, "_mxtmp")
    vocab = json.load(open(files[0]))
    merges = open(files[1]).read().splitlines()
    for f in files:
        os.unlink(f)
    items = sorted(vocab.items(), key=lambda kv: kv[1])
    out = {t: i for i, (t, _) in enumerate(items)}
    # unreachable filler entries keep the GPT-2 vocabulary size (and so the model shape)
    k = 0
    while len(out) < vocab_size - 1:
        out[f"<|mxpad{k}|>"] = len(out)
        k += 1
    out[EOD] = vocab_size - 1
    with open(vocab_file, "w") as f:
        json.dump(out, f, ensure_ascii=False)
    with open(merge_file, "w") as f:
        f.write("#version: 0.2\n")
        for m in merges:
            if m and not m.startswith("#version"):
                f.write(m + "\n")
    return vocab_file, merge_file


class GPT2BPETokenizer:
    def __init__(self, vocab_file: str, merge_file: str):
        from tokenizers import ByteLevelBPETokenizer
        self._tok = ByteLevelBPETokenizer(vocab_file, merge_file, add_prefix_space=False)
        self._vocab = json.load(open(vocab_file))
        self.eod = self._vocab.get(EOD, len(self._vocab) - 1)

    @property
    def vocab_size(self) -> int:
        return len(self._vocab)

    def tokenize(self, text: str) -> List[int]:
        return self._tok.encode(text).ids

    def tokenize_batch(self, texts: List[str]) -> List[List[int]]:
        return [e.ids for e in self._tok.encode_batch(texts)]

    def detokenize(self, ids) -> str:
        return self._tok.decode(list(ids))


class NullTokenizer:
    """`--tokenizer-type NullTokenizer --vocab-size N`: text is whitespace-separated ids."""

    def __init__(self, vocab_size: int):
        self._v = vocab_size
        self.eod = vocab_size - 1

    @property
    def vocab_size(self):
        return self._v

    def tokenize(self, text):
        return [int(x) for x in text.split()]

    def tokenize_batch(self, texts):
        return [self.tokenize(t) for t in texts]

    def detokenize(self, ids):
        return " ".join(str(i) for i in ids)


def build_tokenizer(tokenizer_type: str, vocab_file=None, merge_file=None, vocab_size=None):
    if tokenizer_type in ("GPT2BPETokenizer", "GPT2Tokenizer"):
        return GPT2BPETokenizer(vocab_file, merge_file)
    if tokenizer_type == "NullTokenizer":
        return NullTokenizer(vocab_size)
    raise ValueError(f"tokenizer {tokenizer_type} not supported offline")

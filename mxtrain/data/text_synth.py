"""Synthetic text corpora with the schema of the reference's datasets (the node is
offline):

* ``--style wikicorpus``  JSON lines ``{"id", "title", "text"}`` like HF
  ``load_dataset("wikicorpus", "raw_en").to_json(...)`` (examples/megatron-deepspeed/
  gpt2_345m/wikicorpus.yaml:15-22);
* ``--style redpajama``   JSON lines ``{"text", "meta"}`` like RedPajama ``book.jsonl``
  (charts/machine-learning/data-prep/redpajama-data);
* ``--style mrpc``        TSV/JSON sentence pairs ``{"sentence1","sentence2","label","idx"}``
  (GLUE MRPC shape, for the Accelerate BERT example).

Text is Zipf-distributed pseudo-words (deterministic per seed), so BPE training and
tokenisation behave like natural text statistically.
"""
from __future__ import annotations

import argparse
import json
import os
import random
from typing import List

ONSETS = ["", "b", "c", "d", "f", "g", "h", "k", "l", "m", "n", "p", "r", "s", "t", "v", "w", "st", "tr",
          "pl", "gr", "ch", "sh", "th", "br", "cl"]
VOWELS = ["a", "e", "i", "o", "u", "ea", "ou", "io", "ai"]
CODAS = ["", "n", "r", "s", "t", "l", "m", "nd", "st", "ng", "rt", "ck"]


def lexicon(n: int, seed: int = 0) -> List[str]:
    r = random.Random(seed)
    words, seen = [], set()
    while len(words) < n:
        k = r.choice([1, 1, 2, 2, 2, 3, 3, 4])
        w = "".join(r.choice(ONSETS) + r.choice(VOWELS) + r.choice(CODAS) for _ in range(k))
        if w not in seen:
            seen.add(w)
            words.append(w)
    return words


class TextGen:
    def __init__(self, seed: int = 0, vocab: int = 8000):
        self.r = random.Random(seed)
        self.words = lexicon(vocab, seed=1234)
        # Zipf weights
        self.cum = []
        t = 0.0
        for i in range(len(self.words)):
            t += 1.0 / (i + 1) ** 1.07
            self.cum.append(t)
        self.total = t

    def word(self) -> str:
        import bisect
        return self.words[bisect.bisect_left(self.cum, self.r.random() * self.total)]

    def sentence(self, lo=6, hi=24) -> str:
        n = self.r.randint(lo, hi)
        ws = [self.word() for _ in range(n)]
        if self.r.random() < 0.3:
            ws.insert(self.r.randint(0, n), str(self.r.randint(1, 2025)))
        s = " ".join(ws)
        s = s[0].upper() + s[1:]
        if self.r.random() < 0.2:
            k = self.r.randint(1, n - 1)
            parts = s.split(" ")
            parts[k - 1] += ","
            s = " ".join(parts)
        return s + self.r.choice([".", ".", ".", "!", "?", ";"]) if s[-1] not in ".!?" else s

    def paragraph(self, lo=2, hi=8) -> str:
        return " ".join(self.sentence() for _ in range(self.r.randint(lo, hi)))

    def document(self, lo=2, hi=10) -> str:
        return "\n\n".join(self.paragraph() for _ in range(self.r.randint(lo, hi)))

    def title(self) -> str:
        return " ".join(self.word().capitalize() for _ in range(self.r.randint(1, 4)))


def write_corpus(path: str, num_docs: int, seed: int = 0, style: str = "wikicorpus"):
    g = TextGen(seed)
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    with open(path, "w") as f:
        for i in range(num_docs):
            if style == "wikicorpus":
                rec = {"id": str(i), "title": g.title(), "text": g.document()}
            elif style == "redpajama":
                rec = {"text": g.document(4, 20), "meta": {"title": g.title(), "source": "synthetic",
                                                           "short_book_title": g.title()}}
            elif style == "mrpc":
                s1 = g.sentence(8, 30)
                same = g.r.random() < 0.68
                s2 = s1 if same else g.sentence(8, 30)
                if same:  # paraphrase: perturb a few words
                    ws = s2.split(" ")
                    for _ in range(max(1, len(ws) // 6)):
                        ws[g.r.randrange(len(ws))] = g.word()
                    s2 = " ".join(ws)
                rec = {"sentence1": s1, "sentence2": s2, "label": int(same), "idx": i}
            else:
                raise ValueError(f"unknown style {style}")
            f.write(json.dumps(rec) + "\n")
    return path


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--output", required=True)
    ap.add_argument("--num-docs", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--style", default="wikicorpus", choices=["wikicorpus", "redpajama", "mrpc"])
    a = ap.parse_args(argv)
    write_corpus(a.output, a.num_docs, a.seed, a.style)
    print(f"wrote {a.num_docs} {a.style} records to {a.output}")


if __name__ == "__main__":
    main()

#!/bin/bash
# Offline stand-in for Megatron-DeepSpeed's dataset/download_vocab.sh (which fetches
# gpt2-vocab.json / gpt2-merges.txt from the internet): writes a GPT-2-format byte-level
# BPE vocabulary of the same size (50257, <|endoftext|> = 50256) into the current
# directory, trained on $DATA_ROOT/train.json when present, else on synthetic text.
set -e
PY=${PYTHON:-python3}
# the data-prep job leaves its vocabulary next to the data; reuse it so token ids match
if [[ -n "$DATA_ROOT" && -f "$DATA_ROOT/gpt2-vocab.json" && -f "$DATA_ROOT/gpt2-merges.txt" ]]; then
  cp "$DATA_ROOT/gpt2-vocab.json" "$DATA_ROOT/gpt2-merges.txt" .
  echo "copied gpt2-vocab.json gpt2-merges.txt from $DATA_ROOT"
  exit 0
fi
$PY - <<PYEOF
import json, os
from mxtrain.data.tokenizer import make_gpt2_vocab
src = os.path.join(os.environ.get("DATA_ROOT", ""), "train.json")
corpus = None
if os.path.exists(src):
    corpus = []
    with open(src) as f:
        for i, line in enumerate(f):
            if i >= 20000:
                break
            corpus.append(json.loads(line).get("text", ""))
make_gpt2_vocab("gpt2-vocab.json", "gpt2-merges.txt", corpus)
root = os.environ.get("DATA_ROOT")
if (root and os.path.isdir(root) and os.access(root, os.W_OK)
        and os.path.realpath(root) != os.path.realpath(".")):
    import shutil
    shutil.copy("gpt2-vocab.json", root)
    shutil.copy("gpt2-merges.txt", root)
print("wrote gpt2-vocab.json gpt2-merges.txt (offline byte-level BPE, 50257 entries)")
PYEOF

"""Host-side cost of one eager GPT-2 345M training step: time to enqueue K steps right
after a synchronize (the GPU is still busy with the first ones) vs the synchronized
time of the same K steps.  enqueue/step << gpu/step means the eager step is GPU-bound
(so multi-GPU runs without hipGraph capture have host headroom for the collectives)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.models.gpt import GPT_CONFIGS, GPTConfig  # noqa: E402
from mxtrain.parallel import state as pstate  # noqa: E402
from mxtrain.runtime.gemm_tuning import use_tuned_gemms  # noqa: E402
from mxtrain.training import GPTTrainer, TrainConfig, synthetic_batch  # noqa: E402

torch.backends.cuda.preferred_blas_library("hipblaslt")
use_tuned_gemms()
ps = pstate.initialize_model_parallel()
cfg = GPTConfig(**GPT_CONFIGS["gpt2-345m"])
tr = GPTTrainer(cfg, TrainConfig(micro_batch_size=4), ps)
tok, lab = synthetic_batch(cfg, 1, 4, ps.device)
for _ in range(5):
    tr.train_step(tok, lab)
torch.cuda.synchronize()
K = 10
t0 = time.perf_counter()
for _ in range(K):
    tr.train_step(tok, lab)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(json.dumps({"enqueue_ms_per_step": round((t1 - t0) * 1e3 / K, 3),
                  "gpu_ms_per_step": round((t2 - t0) * 1e3 / K, 3)}))

if os.environ.get("CPU_PROFILE"):
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        tr.train_step(tok, lab)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)

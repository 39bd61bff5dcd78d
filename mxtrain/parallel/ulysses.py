"""Ulysses context parallelism (DeepSpeed-Ulysses, ``--ds-sequence-parallel-size``;
SURVEY §2.6 P8, §5.7): the sequence is split over the ``cp`` ranks of a context-parallel
group for every token-local op (LayerNorm, MLP, dropout, embedding, loss) and re-split
over attention heads around the attention kernel with two all-to-alls:

    [B * S/cp, (H + 2 KV) * D]   local tokens, all heads          (after the QKV GEMM)
        --all-to-all-->  [B * S, (H/cp + 2 KV/cp) * D]   whole sequence, my head group
    flash attention on H/cp heads over the full causal sequence (no K/V exchange)
        --all-to-all-->  [B * S/cp, H * D]   back to local tokens

Token order is token-major everywhere ([b, s] rows), so each all-to-all is one
``all_to_all_single`` of a contiguous [cp, rows, cols] buffer (RCCL over xGMI on GPU,
gloo on CPU) plus one permute copy.  The backward of each exchange is the other one.
On one node every pair of GPUs has its own xGMI link, so the all-to-all uses all 7
links at once, the pattern xGMI is best at.
"""
from __future__ import annotations

from typing import List, Sequence

import torch
import torch.distributed as dist


def _a2a(send: torch.Tensor, group) -> torch.Tensor:
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    return recv


def seq_to_head(x: torch.Tensor, blocks: Sequence[int], B: int, S_local: int, group) -> torch.Tensor:
    """x [B*S_local, sum(blocks)] (column blocks, e.g. Q | K | V, each divisible by cp)
    -> [B*S_local*cp, sum(blocks)/cp]: full sequences, head group ``rank`` of every block."""
    cp = dist.get_world_size(group)
    cols = []
    off = 0
    for w in blocks:
        cols.append((off, w // cp))
        off += w
    # send[j] = my tokens, head group j of every block
    send = torch.stack([torch.cat([x[:, o + j * w:o + (j + 1) * w] for o, w in cols], 1)
                        for j in range(cp)]).contiguous()                     # [cp, T_l, c]
    recv = _a2a(send, group)                                                 # [cp(src seq chunk), T_l, c]
    c = recv.shape[-1]
    return recv.view(cp, B, S_local, c).permute(1, 0, 2, 3).reshape(B * S_local * cp, c)


def head_to_seq(y: torch.Tensor, blocks: Sequence[int], B: int, S_local: int, group) -> torch.Tensor:
    """Inverse of seq_to_head: y [B*S, sum(blocks)/cp] -> [B*S_local, sum(blocks)]."""
    cp = dist.get_world_size(group)
    c = y.shape[-1]
    send = y.view(B, cp, S_local, c).permute(1, 0, 2, 3).reshape(cp, B * S_local, c).contiguous()
    recv = _a2a(send, group)                                                 # [cp(src head grp), T_l, c]
    parts: List[torch.Tensor] = []
    off = 0
    for w in blocks:
        wl = w // cp
        parts += [recv[j][:, off:off + wl] for j in range(cp)]
        off += wl
    return torch.cat(parts, 1)


def local_chunk(t: torch.Tensor, cp: int, cp_rank: int) -> torch.Tensor:
    """[..., S] token ids / labels -> this context-parallel rank's [..., S/cp] slice."""
    S = t.shape[-1]
    assert S % cp == 0, f"sequence length {S} not divisible by context-parallel size {cp}"
    n = S // cp
    return t[..., cp_rank * n:(cp_rank + 1) * n].contiguous()

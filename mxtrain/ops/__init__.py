"""mxtrain.ops -- hand-written CDNA4 (gfx950) HIP kernels bound through ctypes.

GPU tensors always take the HIP path (and raise if the in-tree library is missing);
CPU tensors take the fp32 PyTorch reference path.
"""
from . import _lib  # noqa: F401
from .attention import attn_bwd, attn_fwd, flash_attention  # noqa: F401
from .fused import (bias_gelu, bias_gelu_bwd, bias_gelu_fwd, ce_stats,  # noqa: F401
                    cross_entropy, cross_entropy_fwd_bwd, embed_bwd, embed_fwd, pos_embed_bwd)
from .norm import (bda_norm_fwd, colsum, layer_norm, layernorm_fwd, norm_bwd,  # noqa: F401
                   rms_norm)
from .optim import adamw_step, sumsq_bf16  # noqa: F401
from .rope import apply_rope_, rope  # noqa: F401


def library_loaded() -> bool:
    return _lib._lib is not None


def library_path() -> str:
    return _lib.LIB_PATH

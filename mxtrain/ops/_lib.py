"""ctypes binding of the in-tree HIP kernel library ``mxtrain/lib/libmxkernels.so``.

The library is loaded lazily the first time a GPU op runs.  On a machine with a GPU
the ops never fall back silently: if the library is missing or fails to load, the op
raises (set ``MXTRAIN_ALLOW_TORCH_FALLBACK=1`` to opt into the eager-PyTorch
reference path for debugging).  CPU tensors always use the reference path.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "lib", "libmxkernels.so"))

_lock = threading.Lock()
_lib = None

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
F = ctypes.c_float
U32 = ctypes.c_uint32

# name -> argtypes (every function returns int hipError_t; the stream is the last arg)
SIGNATURES = {
    # norm.hip
    "mx_norm_bwd_nparts": [I],
    "mx_norm_bwd_nparts2": [I, I],
    "mx_flash_qmajor_bk": [I, I],
    "mx_flash_kmajor128_variant": [I],
    # membw.hip (HBM roofline probe, scripts/hbm_probe.py)
    "mx_membw": [I, I, I, P, P, I64, I, P],
    # graph.hip (host-side hipGraph inspection; no stream argument)
    "mx_graph_census": [P, P, I],
    "mx_graph_memsets_to_kernels": [P],
    "mx_layernorm_fwd": [P, P, P, P, P, P, I, I, F, P],
    "mx_rmsnorm_fwd": [P, P, P, P, I, I, F, P],
    "mx_bda_norm_fwd": [P, P, P, P, P, P, P, P, P, I, I, F, F, P, U32, I64, I, P],
    "mx_norm_bwd": [P, P, P, P, P, P, P, P, P, I, I, F, P, U32, I64, I, P],
    "mx_colsum_finalize": [P, I, I, I, P, P, P, I, P, P],
    "mx_colreduce_scratch": [I, I],
    "mx_colsum_bf16": [P, I, I, P, P, I, P],
    "mx_colreduce_batched": [P, I, I, P],
    "mx_colsum_partial_bf16": [P, I, I, P, P],
    # epilogue.hip
    "mx_bias_act_fwd": [P, P, P, I64, I, I, P],
    "mx_bias_act_bwd_parts": [I64, I],
    "mx_bias_act_bwd": [P, P, P, P, P, I64, I, I, I, P],
    # fused.hip
    "mx_bias_gelu_fwd": [P, P, P, I, I, P],
    "mx_bias_gelu_bwd_rows_per_block": [],
    "mx_bias_gelu_bwd": [P, P, P, P, P, I, P, I, I, P],
    "mx_bias_swiglu_fwd": [P, P, P, I, I, P],
    "mx_bias_swiglu_bwd": [P, P, P, P, P, I, P, I, I, P],
    "mx_embed_fwd": [P, P, P, P, I, I, I, I64, I64, I, P],
    "mx_embed_bwd": [P, P, P, P, I, I, I64, I64, P],
    "mx_embed_bwd_scan": [P, P, P, I, I, I64, I64, P],
    "mx_flash_fwd_dgen": [P, P, P, I, I, I, P, I, P, I, I, I, I, I, I, P, F, P, U32, F, I, I, P],
    "mx_pos_embed_bwd": [P, P, I, I, I, P],
    "mx_ce_stats": [P, P, I, I, I64, P, P, P, P],
    "mx_ce_lse": [P, P, P, I, P],
    "mx_ce_grad": [P, P, I, I, I64, P, P, P, P, F, I, P],
    "mx_ce_fused": [P, P, I, I, P, P, F, I, P],
    # detloss.hip
    "mx_detloss_max_blocks": [],
    "mx_rpn_loss_fwd": [P, P, P, P, P, I, F, P, P, P],
    "mx_rpn_loss_bwd": [P, P, P, P, P, I, P, P, P, P, P, P],
    "mx_frcnn_loss_fwd": [P, P, P, P, P, I, I, F, P, P, P],
    "mx_frcnn_loss_bwd": [P, P, P, P, P, I, I, P, P, P, P, P, P],
    "mx_mask_loss_fwd": [P, P, P, P, I, I, I, P, P, P],
    "mx_mask_loss_bwd": [P, P, P, P, I, I, I, P, P, P, P],
    # multitensor.hip
    "mx_mt_chunk": [],
    "mx_mt_max_tensors": [],
    "mx_mt_grad_in": [P, P, P, P, I, P, P, P, P],
    "mx_mt_grad_in_range": [P, P, P, P, I, I, P, P, P, P],
    "mx_mt_scale_sumsq": [P, I64, F, P, P],
    "mx_mt_sumsq_fin": [P, I, P, P],
    "mx_mt_sgd": [P, P, P, I, P, P, P, P, P, P, P],
    "mx_mt_cast": [P, P, P, I, P, P, P],
    # optim.hip
    "mx_sumsq_nparts": [],
    "mx_sumsq_bf16": [P, I64, F, P, P, P, I, P],
    "mx_adamw_step": [P, P, P, P, P, P, I64, P, P, P],
    # flash.hip
    "mx_flash_dropmask": [P, U32, F, I, I, I, I, I, I, P, P, P],
    "mx_flash_dropmask_layers": [P, U32, F, I, I, I, I, I, I, I, P, P, I64, I64, P],
    "mx_flash_fwd": [P, P, P, I, I, I, P, I, P, I, I, I, I, I, I, P, F, P, F, P],
    "mx_flash_bwd": [P, P, P, I, I, I, P, I, P, I, P, P, P, I, P, P, I, I, I, I, I, I, I, I,
                     P, F, P, P, F, P, I, P],
    # gemm.hip
    "mx_gemm_kk_tile": [I, I],
    "mx_gemm_kk": [I, P, I, F, I, I, P, P, P],
    # convwg.hip
    # batchnorm.hip
    "mx_bn_fwd": [P, P, P, P, P, P, P, P, P, I, I, F, F, I, P, P, P, P],
    "mx_bn_apply": [P, P, P, P, P, I, I, I, P],
    "mx_bn2_apply": [P, P, P, P, I, I, P],
    "mx_bn2_bwd": [P, P, P, P, P, P, P, P, P, P, P, I, I, P, P],
    "mx_bn_bwd": [P, P, P, P, P, P, P, P, P, P, I, I, I, I, P, P, I, P],
    "mx_conv_wgrad_tile": [I],
    "mx_conv_wgrad": [P, F, I, P],
    "mx_conv_wgrad_splits": [I64, I],
    "mx_conv_wgrad_reduce_batched": [P, I, P],
    "mx_conv_dgrad": [P, P],
    "mx_conv_fwd": [P, P],
    # gemm_nt.hip
    "mx_gemm_nt_tile": [I, I],
    "mx_gemm_nt": [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, P],
    "mx_gemm_nt_stamps": [P, P, P, P, I, I, I, I, I, I, I, P],
    # rope.hip
    "mx_rope": [P, I64, I, I, I, I, I, I, I, P, P, P, I, P],
    # vision.hip
    "mx_roi_align_fwd": [P, P, P, P, I, I, F, I, P, I, I, I, I, I, I, P, P],
    "mx_roi_align_bwd": [P, P, P, P, I, I, F, I, P, I, I, I, I, I, I, P, P],
    "mx_roi_align_bwd_tiled": [P, P, P, P, I, I, F, I, I, P, I, I, I, I, I, I, P, P, P, P],
    "mx_nms_workspace_words": [I],
    "mx_nms_par": [I],
    "mx_topk_chunk": [],
    "mx_topk_rows": [P, I, I, I, I, I, P, P, P],
    "mx_topk_rows_max_k": [],
    "mx_topk_max_rows": [],
    "mx_level_topk_decode": [P, I, I, P, F, P, P, P, P, I, P, P, P, P],
    "mx_nms": [P, P, I, I, F, I, P, P, P, P],
    "mx_match": [P, I, I, P, P, I, I, P, P, P, P, P],
    "mx_decode_clip": [P, P, I, I, F, F, F, F, F, P, I, P, P],
    "mx_copy_rows": [P, P, I, I, I, I, I64, I64, P],
    "mx_normalize_u8_nhwc": [P, P, I, I, I, P, P, P],
    "mx_stem_pool": [P, P, P, P, I, I, I, P, P, P],
    "mx_crop_resize_masks": [P, I, I, P, P, I, I, P, P],
    "mx_crop_resize_mask_crops": [P, P, I, I, P, P, I, I, P, P],
    "mx_topk_rows_long": [P, I, I, I, I, I, I, I, P, P, P, P, P],
    # dettarget.hip
    "mx_encode_boxes": [P, I, P, I, F, F, F, F, P, P],
    "mx_rpn_keys": [P, I, I, P, P, P, P, P, P, I, F, F, P, P, P, P, P, P],
    "mx_rpn_select": [P, P, I, P, P, I, I, I, I, I, P, P, P],
    "mx_merge_sorted_topk": [P, I, I, I, I, P, P, P],
    "mx_merge_keep_topk": [P, P, P, I, I, I, I, P, P, P],
    "mx_down2_add": [P, P, P, I, I, I, I, P],
    "mx_subsample2": [P, P, I, I, I, I, I, P],
    "mx_maxpool3s2_fwd": [P, P, P, I, I, I, I, P],
    "mx_cast_multi": [P, I, I, P],
    "mx_maxpool3s2_fwd_bn": [P, P, P, I, I, I, I, P, P, P],
    "mx_maxpool3s2_bwd_relu": [P, P, P, P, I, I, I, I, P],
    "mx_gap_fwd": [P, P, I, I, I, P],
    "mx_gap_bwd": [P, P, I, I, I, P],
    "mx_sgd_multi": [P, I, P, F, F, I, P],
    "mx_maxpool3s2_bwd": [P, P, P, I, I, I, I, P],
    "mx_colsum_jobs": [P, I, P],
    "mx_roi_candidates": [P, I, P, P, I, I, P, P, P],
    "mx_roi_fgkey": [P, P, P, I, F, P, P],
    "mx_roi_order": [P, P, I, P, P, P, I, I, F, P, P, P],
    "mx_roi_gather": [P, I, I, I, P, I, P, P, P, P, I, F, F, F, F, P, P, P, P, P, P, P, P],
    "mx_rpn_unpack": [P, I, I, I, I, I, P, I, I, P, P, P],
    "mx_rpn_pack_grad": [P, P, I, I, I, I, I, P, I, I, P, P],
    "mx_add3_nhwc": [P, P, I64, I64, P, P, I, I, I, I, P],
    "mx_rpn_pack": [P, P, P, I, I, I, I, I, P],
    # knobs (one int; return the previous setting)
    "mx_flash_dropmask_variant": [I],
}


def _load():
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"mxtrain HIP kernel library not found at {LIB_PATH}; build it with "
                "`python -m mxtrain.build` (hipcc --offload-arch=gfx950)")
        # torch must be imported first so the process-wide HIP runtime is torch's
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        _lib = lib
        return lib


def lib():
    return _load()


# per-call host cost matters: an eager GPT-2 345M step issues ~1000 launches and its
# Python side was within 20% of the GPU time, so the helpers below avoid torch's
# device/stream bookkeeping and ctypes object churn (raw ints for pointers, cached
# function objects, environment read once)
_FN = {}
_FALLBACK = None


def available() -> bool:
    try:
        _load()
        return True
    except Exception:
        return False


def fallback_allowed() -> bool:
    global _FALLBACK
    if _FALLBACK is None:
        _FALLBACK = os.environ.get("MXTRAIN_ALLOW_TORCH_FALLBACK", "0") == "1"
    return _FALLBACK


def use_hip(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU and the HIP kernels must be used."""
    if not t.is_cuda:
        return False
    if fallback_allowed() and not available():
        return False
    return True


def stream():
    """The current HIP stream of the current device, as a raw handle (int)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def ptr(t):
    if t is None:
        return None
    return t.data_ptr()


def _fn(name):
    f = _FN.get(name)
    if f is None:
        f = _FN[name] = getattr(_load(), name)
    return f


def call(name, *args):
    err = _fn(name)(*args)
    if err != 0:
        raise RuntimeError(f"{name} failed with hipError {err}")
    return err


_QCACHE = {}


def query(name, *args) -> int:
    """Pure size/shape queries of the library (partial counts, scratch sizes): memoised."""
    key = (name,) + args
    v = _QCACHE.get(key)
    if v is None:
        v = _QCACHE[key] = _fn(name)(*args)
    return v


def query64(name, *args) -> int:
    key = (name,) + args
    v = _QCACHE.get(key)
    if v is None:
        fn = _fn(name)
        fn.restype = ctypes.c_int64
        v = _QCACHE[key] = fn(*args)
    return v

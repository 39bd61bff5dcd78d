"""mxtrain -- an MI355X-native (gfx950 / CDNA4) distributed-training launch stack.

Layers: ops (HIP kernels) -> parallel (RCCL DP/TP/PP/SP, ZeRO-1) ->
models (GPT, BERT, Mask R-CNN, ResNet) -> workloads (Megatron / Accelerate / tensorpack /
Ray compatible CLIs) -> runtime + launch (single-node job controllers) -> chart (Helm
values schema + Go-template renderer) -> cli / pipeline.
"""
__version__ = "0.1.0"

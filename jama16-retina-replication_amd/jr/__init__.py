"""jr — MI355X-native engine for the jama16-retina-replication hot path.

Inception-v3 training step and ensemble inference on hand-written gfx950
HIP kernels (libjr.so, C-ABI in include/jr.h).  PyTorch-ROCm provides device
memory, streams and torch.distributed (RCCL); it does no compute here.
"""
__all__ = ["_ffi", "inception", "init", "engine", "dist", "synth"]

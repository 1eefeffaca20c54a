"""ctypes binding of libjr.so (the C-ABI declared in include/jr.h).

This is the only place Python touches the compute library.  Loading is
strict: if libjr.so is missing or was not built for gfx950 the import fails
loudly — there is no CPU or PyTorch fallback for any op on the product path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int32, c_int64,
                    c_size_t, c_uint8, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JR_LIB", os.path.join(_HERE, "libjr.so"))

JR_OK = 0
JR_ERR_INVALID, JR_ERR_HIP, JR_ERR_UNSUPPORTED, JR_ERR_WORKSPACE = -1, -2, -3, -4   # include/jr.h jr_status
JR_ERR_DEVICE = -5   # jr_device_check: a kernel reported a device-side failure
JR_F32 = 0
JR_BF16 = 1
JR_F32_X8 = 2      # conv entry points only: fp32 tensors, bf16x8-split MFMA products (jr.h)
JR_F32_X8P = 3     # conv entry points only: the X8 arithmetic on pre-split h/m/l bf16 operand planes (jr.h)
JR_F32_X6H = 4     # conv entry points only: fp32 tensors, scaled fp16 three-way split, six f16 MFMAs (jr.h)
JR_CONV_FWD, JR_CONV_BWD_DATA, JR_CONV_BWD_FILTER = 0, 1, 2
JR_HEAD_SIGMOID, JR_HEAD_SOFTMAX = 0, 1


class JRError(RuntimeError):
    """A libjr call returned a negative jr_status."""

    def __init__(self, fn: str, status: int, msg: str):
        super().__init__(f"{fn} failed with status {status}: {msg}")
        self.status = status


class ConvDesc(Structure):
    _fields_ = [(n, c_int32) for n in (
        "n", "h", "w", "c_in", "c_out", "kh", "kw", "stride_h", "stride_w", "pad_h", "pad_w",
        "ho", "wo", "x_c_off", "x_c_stride", "y_c_off", "y_c_stride")] + [
        # JR_F32_X6H operand magnitude bounds (jr.h): absmax words or host bounds
        ("x_absmax", c_void_p), ("w_absmax", c_void_p), ("dy_absmax", c_void_p),
        ("x_bound", ctypes.c_float), ("w_bound", ctypes.c_float), ("dy_bound", ctypes.c_float)]


class WPrep(Structure):
    """include/jr.h: struct jr_wprep (one layer of jr_conv_weights_bf16_multi)."""
    _fields_ = [("src_off", c_int64), ("hwio_off", c_int64), ("wt_off", c_int64), ("kh", c_int32),
                ("kw", c_int32), ("c_in", c_int32), ("c_out", c_int32), ("tile_start", c_int32),
                ("reserved", c_int32)]


class AbsmaxSeg(Structure):
    """include/jr.h jr_absmax_seg: one parameter block of jr_absmax_prep."""
    _fields_ = [("off", c_int64), ("count", c_int64), ("out", c_int32), ("limit", c_float)]


class BnSeg(Structure):
    """include/jr.h jr_bn_seg: one member's upstream gradient slice and beta / dbeta."""
    _fields_ = [("dy", c_void_p), ("dy_c_off", c_int32), ("dy_c_stride", c_int32), ("c", c_int32),
                ("beta", c_void_p), ("dbeta", c_void_p)]


class BnApplySeg(Structure):
    """include/jr.h jr_bn_apply_seg: one member's output slice and beta."""
    _fields_ = [("y", c_void_p), ("y_c_off", c_int32), ("y_c_stride", c_int32), ("c", c_int32), ("beta", c_void_p)]


class BnBwdLayer(Structure):
    """include/jr.h jr_bn_bwd_layer: one layer of a batched BN backward."""
    _fields_ = [("nseg", c_int32), ("segs", BnSeg * 4), ("x", c_void_p), ("x_c_off", c_int32),
                ("x_c_stride", c_int32), ("m", c_int64), ("c", c_int32), ("mean", c_void_p),
                ("invstd", c_void_p), ("dx", c_void_p)]


class WgradSeg(Structure):
    """include/jr.h jr_wgrad_seg: one layer of the deferred filter-gradient reduce."""
    _fields_ = [("slabs", c_void_p), ("dw", c_void_p)] + [(n, c_int32) for n in (
        "m", "n", "splits", "c_in", "c_pad", "g", "block0", "blocks")]


class BnPartials(Structure):
    """include/jr.h jr_bn_partials: where a forward GEMM leaves its BN-statistics partials."""
    _fields_ = [("ws_offset", c_int64), ("P", c_int32), ("R", c_int32), ("M", c_int32), ("N", c_int32),
                ("single_stage", c_int32)]


class PoolDesc(Structure):
    _fields_ = [(n, c_int32) for n in (
        "n", "h", "w", "c", "ho", "wo", "x_c_off", "x_c_stride", "y_c_off", "y_c_stride")]


# name -> (restype, argtypes)
_SIGS = {
    "jr_init": (c_int, [c_int]),
    "jr_last_error": (c_char_p, []),
    "jr_version": (c_char_p, []),
    "jr_conv2d_workspace_size": (c_size_t, [POINTER(ConvDesc), c_int, c_int]),
    "jr_conv2d_fwd": (c_int, [POINTER(ConvDesc), c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_size_t, c_void_p]),
    "jr_conv2d_fwd_bn_stats": (c_int, [POINTER(ConvDesc), c_int, c_void_p, c_void_p, c_void_p, c_float,
                                       c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "jr_conv2d_bn_partials_layout": (c_int, [POINTER(ConvDesc), c_int, POINTER(BnPartials)]),
    "jr_conv2d_fwd_bn_partials": (c_int, [POINTER(ConvDesc), c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                          c_void_p]),
    "jr_bn_relu_apply_stats": (c_int, [c_int, c_void_p, c_int32, c_int32, c_int64, c_int32, c_void_p, c_int32, c_int32,
                                       c_int32, c_int32, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                       c_int32, c_void_p]),
    "jr_conv2d_workspace_size_grouped": (c_size_t, [POINTER(ConvDesc), c_int, c_int]),
    "jr_conv2d_fwd_bn_stats_grouped": (c_int, [POINTER(ConvDesc), c_int, c_int, c_void_p, c_int64, c_void_p, c_int64,
                                               c_void_p, c_int64, c_float, c_void_p, c_void_p, c_int64, c_void_p,
                                               c_size_t, c_void_p]),
    "jr_conv2d_bwd_data": (c_int, [POINTER(ConvDesc), c_int, c_void_p, c_void_p, c_void_p, c_int,
                                   c_void_p, c_size_t, c_void_p]),
    "jr_conv2d_bwd_filter": (c_int, [POINTER(ConvDesc), c_int, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_size_t, c_void_p]),
    "jr_conv2d_wgrad_seg": (c_int, [POINTER(ConvDesc), c_int, POINTER(WgradSeg)]),
    "jr_conv2d_bwd_filter_slabs": (c_int, [POINTER(ConvDesc), c_int, c_void_p, c_void_p, c_void_p, c_size_t,
                                           c_void_p]),
    "jr_wgrad_reduce": (c_int, [c_void_p, c_int32, c_int32, c_void_p]),
    "jr_conv2d_autotune": (c_int, [POINTER(ConvDesc), c_int, c_int, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_size_t, c_void_p]),
    "jr_conv2d_get_config": (c_int, [POINTER(ConvDesc), c_int, c_int, c_int]),
    "jr_conv2d_set_config": (c_int, [POINTER(ConvDesc), c_int, c_int, c_int, c_int]),
    "jr_conv2d_config_generation": (ctypes.c_ulonglong, []),
    "jr_conv2d_num_configs": (c_int, [c_int]),
    "jr_conv_weights_bf16_tiles": (c_int32, [c_int32, c_int32, c_int32, c_int32]),
    "jr_conv_weights_bf16": (c_int, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                     c_void_p]),
    "jr_conv_weights_bf16_multi": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                           c_void_p]),
    "jr_conv_weights_x8p": (c_int, [c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                    c_void_p]),
    "jr_conv_weights_x8p_multi": (c_int, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                          c_void_p]),
    "jr_split_x8p": (c_int, [c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p, c_int32, c_int32, c_int32,
                             c_int64, c_void_p]),
    "jr_comm_unique_id": (c_int, [c_void_p]),
    "jr_comm_init": (c_int, [c_int, c_int, c_void_p, c_int, c_void_p]),
    "jr_comm_init_file": (c_int, [c_int, c_int, c_char_p, c_char_p, c_int, c_int, c_void_p]),
    "jr_allreduce_sum": (c_int, [c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    "jr_comm_rank": (c_int, [c_void_p]),
    "jr_comm_world": (c_int, [c_void_p]),
    "jr_comm_destroy": (c_int, [c_void_p]),
    "jr_bn_workspace_size": (c_size_t, [c_int64, c_int32]),
    "jr_bn_relu_bwd_batch_workspace_size": (c_size_t, [c_int32, c_void_p]),
    "jr_bn_relu_apply_multi": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int32, c_int32, c_int64, c_int32,
                                       c_void_p, c_void_p, c_void_p]),
    "jr_bn_relu_bwd_batch": (c_int, [c_int, c_int32, c_void_p, c_void_p, c_size_t, c_void_p]),
    "jr_bn_stats": (c_int, [c_int, c_void_p, c_int64, c_int32, c_float, c_void_p, c_void_p,
                            c_void_p, c_size_t, c_void_p]),
    "jr_bn_relu_apply": (c_int, [c_int, c_void_p, c_int32, c_int32, c_int64, c_int32, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "jr_bn_relu_apply_grouped": (c_int, [c_int, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int64, c_int32,
                                         c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int32, c_int32,
                                         c_int64, c_void_p]),
    "jr_bn_relu_bwd": (c_int, [c_int, c_void_p, c_int32, c_int32, c_void_p, c_int32, c_int32, c_int64, c_int32,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_size_t, c_void_p]),
    "jr_bn_relu_bwd_multi": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int32, c_int32, c_int64, c_int32,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "jr_bn_relu_bwd_multi_absmax": (c_int, [c_int, c_int, c_void_p, c_void_p, c_int32, c_int32, c_int64, c_int32,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
    "jr_absmax_prep": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_void_p]),
    "jr_maxpool3x3s2_fwd": (c_int, [POINTER(PoolDesc), c_int, c_void_p, c_void_p, c_void_p,
                                    c_void_p]),
    "jr_bn_relu_maxpool3x3s2_fwd": (c_int, [POINTER(PoolDesc), c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p]),
    "jr_bn_relu_bwd_maxpool_workspace_size": (c_size_t, [POINTER(PoolDesc)]),
    "jr_bn_relu_bwd_maxpool": (c_int, [c_int, POINTER(PoolDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                       c_void_p]),
    "jr_bn_relu_bwd_maxpool_absmax": (c_int, [c_int, POINTER(PoolDesc), c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_size_t, c_void_p, c_void_p]),
    "jr_bn_relu_maxpool3x3s2_fwd_grouped": (c_int, [POINTER(PoolDesc), c_int, c_int32, c_void_p, c_void_p, c_void_p,
                                                    c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "jr_maxpool3x3s2_bwd": (c_int, [POINTER(PoolDesc), c_int, c_void_p, c_void_p, c_void_p, c_int,
                                    c_void_p]),
    "jr_avgpool3x3s1_fwd": (c_int, [POINTER(PoolDesc), c_int, c_void_p, c_void_p, c_void_p]),
    "jr_avgpool3x3s1_bwd": (c_int, [POINTER(PoolDesc), c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "jr_gap_fwd": (c_int, [c_int, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "jr_gap_bwd": (c_int, [c_int, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "jr_head_fwd": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                            c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "jr_head_bwd": (c_int, [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                            c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "jr_nesterov_update": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float,
                                   c_float, c_void_p]),
    "jr_momentum_update": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float,
                                   c_float, c_void_p]),
    "jr_sgd_update": (c_int, [c_void_p, c_void_p, c_int64, c_float, c_float, c_void_p]),
    "jr_adam_update": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float,
                               c_float, c_float, c_float, c_void_p]),
    "jr_cast_f32_to_bf16": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "jr_cast_bf16_to_f32": (c_int, [c_void_p, c_void_p, c_int64, c_void_p]),
    "jr_u8_to_f32_scaled": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_void_p]),
    "jr_image_u8_to_nhwc": (c_int, [c_void_p, c_void_p, c_int, c_int64, c_int32, c_int32, c_void_p]),
    "jr_brier_accumulate": (c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "jr_crc32c": (ctypes.c_uint32, [c_void_p, c_size_t, ctypes.c_uint32]),
    "jr_masked_crc32c": (ctypes.c_uint32, [c_void_p, c_size_t]),
    "jr_tfrecord_index": (c_int, [c_void_p, c_size_t, c_int, c_void_p, c_void_p, c_size_t, c_void_p]),
    "jr_example_parse_image": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p]),
    "jr_graph_begin": (c_int, [c_void_p]),
    "jr_graph_end": (c_int, [c_void_p, POINTER(c_void_p)]),
    "jr_graph_launch": (c_int, [c_void_p, c_void_p]),
    "jr_graph_destroy": (c_int, [c_void_p]),
    "jr_graph_regions": (c_int, [c_void_p]),
    "jr_event_create": (c_int, [ctypes.POINTER(c_void_p)]),
    "jr_event_record": (c_int, [c_void_p, c_void_p]),
    "jr_stream_wait_event": (c_int, [c_void_p, c_void_p]),
    "jr_event_destroy": (c_int, [c_void_p]),
    "jr_device_check": (c_int, []),
    "jr_debug_poison_sk_counts": (c_int, [c_void_p, ctypes.c_uint32]),
}

EXPORTED = tuple(_SIGS)

_lib = None


def load() -> ctypes.CDLL:
    """Load libjr.so once; raise if it is absent (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    diag = os.environ.get("JR_LIB_DIAG")    # diagnostic builds only (e.g. libjr_stamps.so, `make stamps`)
    if diag:
        lib = ctypes.CDLL(diag)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libjr.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; "
            "g.build()'` (hipcc --offload-arch=gfx950); the jr path has no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


# host-only entry points (TFRecord / Example parsing, CRC32C, the error text):
# no GPU involved; JR_HOST_LIB may point them at another build of the same
# sources, e.g. the AddressSanitizer build (`make asan`, tests/test_asan_host.py)
HOST_FUNCS = ("jr_last_error", "jr_crc32c", "jr_masked_crc32c", "jr_tfrecord_index", "jr_example_parse_image")
_host = None


def load_host() -> ctypes.CDLL:
    global _host
    if _host is not None:
        return _host
    path = os.environ.get("JR_HOST_LIB")
    if not path:
        _host = load()
        return _host
    lib = ctypes.CDLL(path)
    for name in HOST_FUNCS:
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = _SIGS[name]
    _host = lib
    return lib


def host_last_error() -> str:
    return load_host().jr_last_error().decode(errors="replace")


def last_error() -> str:
    return load().jr_last_error().decode(errors="replace")


def check(name: str, rc: int) -> None:
    if rc != JR_OK:
        raise JRError(name, rc, last_error())


def device_check() -> None:
    """jr_device_check on the current device (after the caller synchronised
    its streams): raise JRError when a stream-K hand-off count word was not
    left zero (counted past its piece count by a launch, or found stale on an
    idle stream); the library has then reset its hand-off words, so later
    launches are correct again."""
    check("jr_device_check", load().jr_device_check())


def call(name: str, *args) -> int:
    lib = load()
    rc = getattr(lib, name)(*args)
    if isinstance(rc, int) and name not in ("jr_conv2d_workspace_size", "jr_bn_workspace_size",
                                            "jr_bn_relu_bwd_maxpool_workspace_size",
                                            "jr_conv2d_get_config", "jr_conv2d_num_configs", "jr_conv2d_config_generation",
                                            "jr_conv_weights_bf16_tiles"):
        check(name, rc)
    return rc


_inited = set()


def init(device: int) -> None:
    """jr_init: select the device and verify it is gfx950."""
    if device in _inited:
        return
    check("jr_init", load().jr_init(device))
    _inited.add(device)

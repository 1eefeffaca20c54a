"""The C-ABI library loads without a GPU and exports every entry point
include/jr.h declares; argument validation runs before any HIP call."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def header_symbols(name="jr.h"):
    text = open(os.path.join(ROOT, "include", name)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(jr_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_hot_path_surface():
    syms = header_symbols()
    for s in ("jr_conv2d_fwd", "jr_conv2d_bwd_data", "jr_conv2d_bwd_filter", "jr_bn_stats", "jr_bn_relu_apply",
              "jr_bn_relu_bwd", "jr_maxpool3x3s2_fwd", "jr_bn_relu_maxpool3x3s2_fwd", "jr_bn_relu_bwd_maxpool", "jr_bn_relu_maxpool3x3s2_fwd_grouped", "jr_avgpool3x3s1_bwd", "jr_gap_fwd", "jr_head_fwd",
              "jr_head_bwd", "jr_nesterov_update", "jr_sgd_update", "jr_graph_begin", "jr_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from jr import _ffi
    lib = ctypes.CDLL(_ffi.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes binding covers the same surface
    assert set(_ffi.EXPORTED) >= set(header_symbols()) - {"jr_conv2d_debug_time"}


def test_jpeg_library_exports_every_declared_symbol():
    """include/jr_jpeg.h -> libjr_jpeg.so (host-only, built by the same Makefile)."""
    from jr import jpeg
    assert jpeg.available(), "libjr_jpeg.so not built"
    lib = ctypes.CDLL(jpeg.LIB_PATH)
    syms = header_symbols("jr_jpeg.h")
    assert {"jr_jpeg_header", "jr_jpeg_decode", "jr_jpeg_last_error"} <= set(syms)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_validation_errors_without_gpu():
    from jr import _ffi
    L = _ffi.load()
    assert L.jr_conv2d_fwd(None, 0, None, None, None, None, 0, None) == -1
    assert "null descriptor" in _ffi.last_error()
    d = _ffi.ConvDesc(1, 8, 8, 16, 16, 3, 3, 1, 1, 1, 1, 9, 8, 0, 16, 0, 16)
    assert L.jr_conv2d_fwd(ctypes.byref(d), 0, 16, 16, 16, None, 0, None) == -1
    assert "ho/wo" in _ffi.last_error()
    d = _ffi.ConvDesc(1, 8, 8, 16, 24, 3, 3, 1, 1, 1, 1, 8, 8, 0, 16, 0, 24)
    assert L.jr_conv2d_fwd(ctypes.byref(d), 0, 16, 16, 16, None, 0, None) == -3   # c_out % 16
    assert L.jr_conv2d_workspace_size(None, 0, 0) == 0
    # JR_F32_X8 (dtype 2): fp32 storage rules and tile table, conv entry points only
    d = _ffi.ConvDesc(2, 17, 17, 64, 96, 3, 3, 1, 1, 1, 1, 17, 17, 0, 64, 0, 96)
    # (x8 ids 0-13: the split kernel; 14-27: the fp32-MFMA kernel of the same
    # tiles; 28-41: the stream-K grid of the split kernel, whose hand-off slots
    # need more workspace)
    assert L.jr_conv2d_num_configs(2) == 3 * L.jr_conv2d_num_configs(0) > 0
    for op in range(3):
        assert L.jr_conv2d_workspace_size(ctypes.byref(d), op, 2) >= L.jr_conv2d_workspace_size(ctypes.byref(d), op, 0)
    # JR_F32_X8P (dtype 3): bf16-operand channel rules (radix 8), its own tile table
    assert L.jr_conv2d_num_configs(3) > 0
    assert L.jr_conv2d_workspace_size(ctypes.byref(d), 0, 3) > 0
    d4 = _ffi.ConvDesc(2, 17, 17, 68, 96, 3, 3, 1, 1, 1, 1, 17, 17, 0, 68, 0, 96)
    assert L.jr_conv2d_fwd(ctypes.byref(d4), 3, 16, 16, 16, None, 0, None) == -1     # strides % 8
    # JR_F32_X6H (dtype 4): the JR_F32_X8 id space and workspaces, conv entry points only
    assert L.jr_conv2d_num_configs(4) == L.jr_conv2d_num_configs(2)
    for op in range(3):
        assert L.jr_conv2d_workspace_size(ctypes.byref(d), op, 4) == L.jr_conv2d_workspace_size(ctypes.byref(d), op, 2)
    assert L.jr_bn_relu_apply(4, 16, 0, 8, 10, 8, 16, 16, 16, 16, 0, 8, None) == -1   # x6h is conv-only
    assert L.jr_conv2d_num_configs(5) == 0
    assert L.jr_conv2d_fwd(ctypes.byref(d), 5, 16, 16, 16, None, 0, None) == -1      # bad dtype
    assert L.jr_absmax_prep(None, None, 0, None, 0, None) == -1
    assert L.jr_split_x8p(16, 10, 6, 0, 4, 16, 8, 0, 8, 80, None) == -1              # slice past src stride
    assert L.jr_split_x8p(16, 10, 4, 0, 4, 16, 8, 0, 8, 40, None) == -1              # planes overlap
    assert L.jr_bn_relu_apply(2, 16, 0, 8, 10, 8, 16, 16, 16, 16, 0, 8, None) == -1   # x8 is conv-only
    assert L.jr_bn_relu_apply(0, 16, 0, 6, 10, 6, 16, 16, 16, 16, 0, 6, None) == -1   # c % 4
    assert L.jr_bn_relu_apply(0, 16, 4, 8, 10, 8, 16, 16, 16, 16, 0, 8, None) == -1   # x slice out of range
    assert L.jr_head_fwd(0, None, None, None, None, 1, 1, 1, None, None, None, None) == -1
    assert L.jr_graph_launch(None, None) == -1


def test_crc32c_known_answers():
    from jr import tfrecord
    assert tfrecord.crc32c(b"123456789") == 0xE3069283          # CRC-32C check value
    assert tfrecord.crc32c(b"") == 0
    assert tfrecord.crc32c(bytes(32)) == 0x8A9136AA             # RFC 3720 B.4: 32 zero bytes
    assert tfrecord.crc32c(bytes([0xFF] * 32)) == 0x62A8AB43    # RFC 3720 B.4: 32 0xff bytes
    c = tfrecord.crc32c(b"123456789")
    assert tfrecord.masked_crc32c(b"123456789") == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    from jr import _ffi
    monkeypatch.setattr(_ffi, "_lib", None)
    monkeypatch.setattr(_ffi, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.delenv("JR_LIB_DIAG", raising=False)
    with pytest.raises(ImportError):
        _ffi.load()
    # (monkeypatch restores _lib and LIB_PATH; no module reload, which would
    # leave the restored library bound to the old module's ctypes classes)

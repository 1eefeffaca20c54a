"""Host-side guards that need no GPU (argument checks run before any HIP call):

* jr_conv2d_config_generation moves only when an override CHANGES, and
  jr_conv2d_bwd_filter_slabs refuses a slab region whose size no longer
  matches the plan (a deferred filter-gradient segment bound to
  an older split count would otherwise sum stale slabs silently);
* jr_comm_init_file ignores an id file another job left at the path (a
  different run id) instead of joining it."""
import ctypes
import struct

import pytest

JR_ERR_INVALID = -1   # include/jr.h jr_status


def _wgrad_desc():
    from jr import _ffi
    # 17^2 1x7 192 -> 192 at B = 64: the filter-gradient GEMM splits K
    return _ffi.ConvDesc(64, 17, 17, 192, 192, 1, 7, 1, 1, 0, 3, 17, 17, 0, 192, 0, 192)


def test_config_generation_moves_only_on_change():
    from jr import _ffi
    L = _ffi.load()
    d = _wgrad_desc()
    wg = _ffi.JR_CONV_BWD_FILTER
    _ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), wg, _ffi.JR_BF16, 0, -1))
    g0 = L.jr_conv2d_config_generation()
    _ffi.check("reset again", L.jr_conv2d_set_config(ctypes.byref(d), wg, _ffi.JR_BF16, 0, -1))
    assert L.jr_conv2d_config_generation() == g0                 # nothing changed
    _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), wg, _ffi.JR_BF16, 0, 3 | (4 << 8)))
    g1 = L.jr_conv2d_config_generation()
    assert g1 > g0
    _ffi.check("set same", L.jr_conv2d_set_config(ctypes.byref(d), wg, _ffi.JR_BF16, 0, 3 | (4 << 8)))
    assert L.jr_conv2d_config_generation() == g1                 # equal value: no bump
    _ffi.check("reset", L.jr_conv2d_set_config(ctypes.byref(d), wg, _ffi.JR_BF16, 0, -1))
    assert L.jr_conv2d_config_generation() > g1


def test_slab_launch_refuses_a_changed_plan():
    from jr import _ffi
    L = _ffi.load()
    d = _wgrad_desc()
    wg = _ffi.JR_CONV_BWD_FILTER
    try:
        _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), wg, _ffi.JR_BF16, 0, 3 | (8 << 8)))
        seg = _ffi.WgradSeg()
        _ffi.check("seg", L.jr_conv2d_wgrad_seg(ctypes.byref(d), _ffi.JR_BF16, ctypes.byref(seg)))
        assert seg.splits == 8
        nb = 4 * seg.splits * seg.m * seg.n
        # another caller re-plans the same geometry with fewer splits
        _ffi.check("set", L.jr_conv2d_set_config(ctypes.byref(d), wg, _ffi.JR_BF16, 0, 3 | (4 << 8)))
        fake = ctypes.c_void_p(1 << 20)          # never dereferenced: the check fails first
        rc = L.jr_conv2d_bwd_filter_slabs(ctypes.byref(d), _ffi.JR_BF16, fake, fake, fake, nb, None)
        assert rc == JR_ERR_INVALID and "slab bytes differ" in _ffi.last_error()
    finally:
        L.jr_conv2d_set_config(ctypes.byref(d), wg, _ffi.JR_BF16, 0, -1)


def test_comm_id_file_of_another_run_is_ignored(tmp_path):
    from jr import _ffi
    L = _ffi.load()
    path = tmp_path / "uid"
    # a complete id file of an earlier job (run "old"), in the jr_comm format
    path.write_bytes(b"JRCOMMID" + struct.pack("<I", 3) + b"old" + bytes(128))
    h = ctypes.c_void_p()
    rc = L.jr_comm_init_file(1, 2, str(path).encode(), b"new", 0, 300, ctypes.byref(h))
    assert rc == JR_ERR_INVALID and "timed out" in _ffi.last_error() and not h.value
    # no run id at all is refused up front
    rc = L.jr_comm_init_file(1, 2, str(path).encode(), b"", 0, 300, ctypes.byref(h))
    assert rc == JR_ERR_INVALID and "run_id" in _ffi.last_error()


def test_jrcomm_requires_a_run_id(monkeypatch, tmp_path):
    from jr.dist import JrComm
    for k in ("TORCHELASTIC_RUN_ID", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(ValueError, match="run_id"):
        JrComm(1, 2, 0, uid_path=str(tmp_path / "uid"))

"""The drop-in boundary: libjmhip.so loads on CPU, exports every entry point include/jmhip.h
declares, and reports errors through status codes (no compute without a GPU)."""
import ctypes
import re

import pytest

from jmpaths import HEADER, LIBJMHIP, ensure_built, load_jmhip

jmhip = load_jmhip()


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(jmh_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    ensure_built()
    lib = ctypes.CDLL(LIBJMHIP)
    names = declared()
    assert len(names) == 37
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(jmhip.EXPORTED)


def test_version_and_strerror():
    lib = jmhip.load()
    assert lib.jmh_abi_version() == jmhip.JMH_ABI_VERSION == 14
    for code, text in jmhip.STATUS.items():
        assert lib.jmh_strerror(code).decode() == text


def test_invalid_config_rejected_before_device_use():
    lib = jmhip.load()
    ctx = ctypes.c_void_p()
    bad = jmhip.make_config(100, 64)                      # width not a multiple of 16
    assert lib.jmh_create(ctypes.byref(bad), 0, ctypes.byref(ctx)) == -1
    bad = jmhip.make_config(64, 64, search_range=0)
    assert lib.jmh_create(ctypes.byref(bad), 0, ctypes.byref(ctx)) == -1
    unsup = jmhip.make_config(64, 64, search_range=48)     # beyond the LDS-resident window
    assert lib.jmh_create(ctypes.byref(unsup), 0, ctypes.byref(ctx)) == -4
    assert lib.jmh_create(None, 0, ctypes.byref(ctx)) == -1


def test_no_device_fails_loudly():
    lib = jmhip.load()
    if lib.jmh_device_count() > 0:
        pytest.skip("a HIP device is present")
    ctx = ctypes.c_void_p()
    cfg = jmhip.make_config(64, 64, search_range=8)
    assert lib.jmh_create(ctypes.byref(cfg), 0, ctypes.byref(ctx)) == -6
    with pytest.raises(jmhip.JmhError):
        jmhip.Encoder(64, 64, search_range=8)


def test_null_context_calls_are_rejected():
    lib = jmhip.load()
    assert lib.jmh_frame_wait(None) == -1
    assert lib.jmh_sync(None) == -1
    assert not lib.jmh_get_mb_result(None, 0)
    lib.jmh_destroy(None)


def test_result_layout_matches_header():
    # jmh_mb_result is 924 bytes with the documented field offsets (numpy mirror == C layout)
    d = jmhip.MB_RESULT_DTYPE
    assert d.itemsize == 924
    assert (d.fields["mv"][1], d.fields["luma"][1], d.fields["chroma_ac"][1], d.fields["min_cost"][1]) == (36, 100, 660, 916)

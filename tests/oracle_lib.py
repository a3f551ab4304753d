"""ctypes binding of the oracle (oracle/_build/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Mirrors jmhip.Encoder so parity tests read the same on both sides.
"""
import ctypes

import numpy as np

from jmpaths import LIBORACLE, ensure_built, load_jmhip

jmhip = load_jmhip()
_P, _I = ctypes.c_void_p, ctypes.c_int
_lib = None


def lib():
    global _lib
    if _lib is None:
        ensure_built()
        L = ctypes.CDLL(LIBORACLE)
        sig = {
            "jmo_create": (_I, [ctypes.POINTER(jmhip.JmhConfig), ctypes.POINTER(_P)]),
            "jmo_destroy": (None, [_P]),
            "jmo_set_reference": (_I, [_P, _P, _P, _P, _I, _I]),
            "jmo_set_reference_u16": (_I, [_P, _P, _P, _P, _I, _I]),
            "jmo_encode_frame_u16": (_I, [_P, _P, _P, _P, _I, _I, ctypes.POINTER(jmhip.JmhFrameParams)]),
            "jmo_read_recon_u16": (_I, [_P, _P, _P, _P, _I, _I]),
            "jmo_encode_frame": (_I, [_P, _P, _P, _P, _I, _I, ctypes.POINTER(jmhip.JmhFrameParams)]),
            "jmo_mb_result": (_P, [_P, _I]),
            "jmo_read_recon": (_I, [_P, _P, _P, _P, _I, _I]),
            "jmo_read_qpel": (_I, [_P, _P]),
            "jmo_load_current": (_I, [_P, _P, _P, _P, _I, _I]),
            "jmo_ffs_sad_table": (_I, [_P, _I, _P, _P, _P]),
            "jmo_tq4x4_batch": (_I, [_I, _P, _P, _I, _I, _P, _P, _P, _P]),
            "jmo_tq8x8_batch": (_I, [_I, _P, _P, _I, _I, _P, _P, _P, _P]),
            "jmo_forward8x8": (None, [_P, _P]),
            "jmo_inverse8x8": (None, [_P, _P]),
            "jmo_satd8x8": (_I, [_P, _I]),
            "jmo_intra8x8_pred": (_I, [_P, _I, _P]),
            "jmo_luma_qpel_sample": (_I, [_P, _I, _I, _I, _I, _I]),
            "jmo_spiral": (None, [_I, _P, _P]),
            "jmo_mvbits": (_I, [_I]),
            "jmo_satd4x4": (_I, [_P, _I]),
            "jmo_forward4x4": (None, [_P, _P]),
            "jmo_inverse4x4": (None, [_P, _P]),
            "jmo_qp2quant": (_I, [_I]),
            "jmo_qp_scale_cr": (_I, [_I]),
            "jmo_mvp_median": (None, [_I] * 17 + [_P]),
            "jmo_search_pictures": (_I, [_P, _P, _P, _I]),
            "jmo_block_motion_search": (_I, [_P, _I, _P, _P]),
            "jmo_hbd_create": (_I, [_I, _I, _I, ctypes.POINTER(_P)]),
            "jmo_hbd_destroy": (None, [_P]),
            "jmo_hbd_pictures": (_I, [_P, _P, _P, _I, _I]),
            "jmo_hbd_qpel": (_I, [_P, _I, _I]),
            "jmo_hbd_block_motion_search": (_I, [_P, _I, _I, _P, _P]),
            "jmo_hbd_sad_table": (_I, [_P, _I, _P, _P, _P]),
            "jmo_hbd_tq4x4_batch": (_I, [_I, _P, _P, _I, _I, _I, _P, _P, _P, _P]),
            "jmo_hbd_tq8x8_batch": (_I, [_I, _P, _P, _I, _I, _I, _P, _P, _P, _P]),
            "jmo_dec_create": (_I, [ctypes.POINTER(_P)]),
            "jmo_dec_destroy": (None, [_P]),
            "jmo_decode_annexb": (_I, [_P, _P, ctypes.c_long, _P, ctypes.c_long, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
            "jmo_dec_error": (ctypes.c_char_p, [_P]),
            "jmo_dec_bit_depth": (_I, [_P]),
        }
        for n, (r, a) in sig.items():
            f = getattr(L, n)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleEncoder:
    def __init__(self, width, height, **kw):
        self.L = lib()
        self.w, self.h = width, height
        self.mbw, self.mbh = width // 16, height // 16
        self.cfg = jmhip.make_config(width, height, **kw)
        self.sfx = "_u16" if self.cfg.bit_depth > 8 else ""          # High 10: 16-bit pictures
        self.pdt = np.uint16 if self.cfg.bit_depth > 8 else np.uint8
        c = ctypes.c_void_p()
        st = self.L.jmo_create(ctypes.byref(self.cfg), ctypes.byref(c))
        if st:
            raise RuntimeError(f"jmo_create: {st}")
        self.ctx = c

    def close(self):
        if self.ctx:
            self.L.jmo_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_reference(self, y, u, v):
        y, u, v = (np.ascontiguousarray(a, self.pdt) for a in (y, u, v))
        assert getattr(self.L, "jmo_set_reference" + self.sfx)(self.ctx, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2) == 0

    def load_current(self, y, u, v):
        assert self.L.jmo_load_current(self.ctx, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2) == 0

    def encode(self, y, u, v, slice_type, qp, chroma_qp_offset=0):
        fp = jmhip.frame_params(slice_type, qp, chroma_qp_offset, rdo=self.cfg.rdo, bit_depth=self.cfg.bit_depth)
        y, u, v = (np.ascontiguousarray(a, self.pdt) for a in (y, u, v))
        st = getattr(self.L, "jmo_encode_frame" + self.sfx)(self.ctx, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2,
                                                           ctypes.byref(fp))
        assert st == 0, st
        n = self.mbw * self.mbh
        p = self.L.jmo_mb_result(self.ctx, 0)
        buf = (ctypes.c_char * (n * jmhip.MB_RESULT_DTYPE.itemsize)).from_address(p)
        res = np.frombuffer(bytes(buf), dtype=jmhip.MB_RESULT_DTYPE).copy()
        ry = np.empty((self.h, self.w), self.pdt)
        ru = np.empty((self.h // 2, self.w // 2), self.pdt)
        rv = np.empty_like(ru)
        assert getattr(self.L, "jmo_read_recon" + self.sfx)(self.ctx, _ptr(ry), _ptr(ru), _ptr(rv), self.w, self.w // 2) == 0
        return res, (ry, ru, rv)

    def read_qpel(self):
        out = np.empty((16, self.h + 8, self.w + 8), np.uint8)
        assert self.L.jmo_read_qpel(self.ctx, _ptr(out)) == 0
        return out

    def search_pictures(self, cur_y, ref_y):
        cur_y, ref_y = np.ascontiguousarray(cur_y, np.uint8), np.ascontiguousarray(ref_y, np.uint8)
        assert self.L.jmo_search_pictures(self.ctx, _ptr(cur_y), _ptr(ref_y), self.w) == 0

    def block_motion_search(self, reqs):
        out = (jmhip.JmhBlockResult * len(reqs))()
        st = self.L.jmo_block_motion_search(self.ctx, len(reqs), ctypes.cast(reqs, _P), ctypes.cast(out, _P))
        assert st == 0, st
        return out

    def sad_table(self, mb_xy, centres):
        mb_xy = np.ascontiguousarray(mb_xy, np.int32)
        centres = np.ascontiguousarray(centres, np.int32)
        side = 2 * self.cfg.search_range + 1
        out = np.empty((mb_xy.shape[0], 16, side * side), np.uint16)
        assert self.L.jmo_ffs_sad_table(self.ctx, mb_xy.shape[0], _ptr(mb_xy), _ptr(centres), _ptr(out)) == 0
        return out


def tq4x4(resid, pred, qp, intra):
    L = lib()
    resid = np.ascontiguousarray(resid, np.int16)
    pred = np.ascontiguousarray(pred, np.uint8)
    n = resid.shape[0]
    lev = np.empty((n, 16), np.int16)
    rec = np.empty((n, 16), np.uint8)
    cc = np.empty(n, np.int32)
    nz = np.empty(n, np.int32)
    assert L.jmo_tq4x4_batch(n, _ptr(resid), _ptr(pred), qp, intra, _ptr(lev), _ptr(rec), _ptr(cc), _ptr(nz)) == 0
    return lev, rec, cc, nz


def tq8x8(resid, pred, qp, intra):
    L = lib()
    resid = np.ascontiguousarray(resid, np.int16)
    pred = np.ascontiguousarray(pred, np.uint8)
    n = resid.shape[0]
    lev = np.empty((n, 64), np.int16)
    rec = np.empty((n, 64), np.uint8)
    cc = np.empty(n, np.int32)
    nz = np.empty(n, np.int32)
    assert L.jmo_tq8x8_batch(n, _ptr(resid), _ptr(pred), qp, intra, _ptr(lev), _ptr(rec), _ptr(cc), _ptr(nz)) == 0
    return lev, rec, cc, nz


def decode_annexb(data, max_frames=64, max_w=1920, max_h=1088):
    L = lib()
    d = ctypes.c_void_p()
    L.jmo_dec_create(ctypes.byref(d))
    buf = np.frombuffer(data, np.uint8).copy()
    cap = max_frames * max_w * max_h * 3   # room for 16-bit samples (High 10)
    out = np.empty(cap, np.uint8)
    w, h = ctypes.c_int(), ctypes.c_int()
    n = L.jmo_decode_annexb(d, _ptr(buf), len(buf), _ptr(out), cap, ctypes.byref(w), ctypes.byref(h))
    err = L.jmo_dec_error(d).decode()
    bd = L.jmo_dec_bit_depth(d)
    L.jmo_dec_destroy(d)
    if n < 0:
        raise RuntimeError("decode failed: " + err)
    fs = w.value * h.value * 3 // 2
    if bd > 8:   # 16-bit LE samples
        o16 = out[:n * fs * 2].view("<u2")
        return [o16[i * fs:(i + 1) * fs] for i in range(n)], w.value, h.value
    return [out[i * fs:(i + 1) * fs] for i in range(n)], w.value, h.value


class OracleHbd:
    """The High 10 per-block seams of the oracle (oracle/hbd.c): the checker of jmh_*_u16."""

    def __init__(self, width, height, search_range, use_hadamard=1):
        self.L = lib()
        self.w, self.h, self.sr, self.had = width, height, search_range, use_hadamard
        h = _P()
        assert self.L.jmo_hbd_create(width, height, search_range, ctypes.byref(h)) == 0
        self.h_ = h

    def close(self):
        if self.h_:
            self.L.jmo_hbd_destroy(self.h_)
            self.h_ = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def pictures(self, cur_y, ref_y, bit_depth):
        cur_y, ref_y = np.ascontiguousarray(cur_y, np.uint16), np.ascontiguousarray(ref_y, np.uint16)
        assert self.L.jmo_hbd_pictures(self.h_, _ptr(cur_y), _ptr(ref_y), self.w, bit_depth) == 0

    def qpel(self, X, Y):
        return self.L.jmo_hbd_qpel(self.h_, X, Y)

    def block_motion_search(self, reqs):
        out = (jmhip.JmhBlockResult * len(reqs))()
        st = self.L.jmo_hbd_block_motion_search(self.h_, self.had, len(reqs), ctypes.cast(reqs, _P), ctypes.cast(out, _P))
        assert st == 0, st
        return out

    def sad_table(self, mb_xy, centres):
        mb_xy = np.ascontiguousarray(mb_xy, np.int32)
        centres = np.ascontiguousarray(centres, np.int32)
        side = 2 * self.sr + 1
        out = np.empty((mb_xy.shape[0], 16, side * side), np.uint16)
        assert self.L.jmo_hbd_sad_table(self.h_, mb_xy.shape[0], _ptr(mb_xy), _ptr(centres), _ptr(out)) == 0
        return out


def tq_u16(resid, pred, qp, intra, bit_depth):
    """jmo_hbd_tq4x4_batch (resid[n][16]) / jmo_hbd_tq8x8_batch (resid[n][64])."""
    L = lib()
    resid = np.ascontiguousarray(resid, np.int16)
    pred = np.ascontiguousarray(pred, np.uint16)
    n, el = resid.shape
    lev = np.empty((n, el), np.int16)
    rec = np.empty((n, el), np.uint16)
    cc = np.empty(n, np.int32)
    nz = np.empty(n, np.int32)
    fn = L.jmo_hbd_tq4x4_batch if el == 16 else L.jmo_hbd_tq8x8_batch
    assert fn(n, _ptr(resid), _ptr(pred), qp, intra, bit_depth, _ptr(lev), _ptr(rec), _ptr(cc), _ptr(nz)) == 0
    return lev, rec, cc, nz

"""CABAC tables (host/cabac.c, SymbolMode 1) against properties of their derivation in ITU-T H.264
9.3.3.2: the LPS probability of state s is p_s = 0.5 * alpha^s, alpha = (0.01875 / 0.5)^(1/63);
rangeTabLPS[s][q] ~ p_s * (288 + 64 q) (the mid-point of range quarter q) and transIdxLPS[s] ~ the
state of alpha * p_s + (1 - alpha) (the LPS update).  The (m, n) initialisation values cannot be
derived; every context the encoder codes must have one (the closed-loop tests decode them with
the independent decoder's own copy of the tables)."""
import ctypes
import math

import numpy as np

from jmpaths import LIBJMHOST, ensure_built

ALPHA = (0.01875 / 0.5) ** (1 / 63)


def lib():
    ensure_built()
    h = ctypes.CDLL(LIBJMHOST)
    for f in ("jm_cabac_range_lps", "jm_cabac_trans_lps", "jm_cabac_init_table"):
        getattr(h, f).restype = ctypes.c_void_p
    return h


def arr(ptr, n, ct, dt):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), (n,)).astype(dt)


def test_range_lps_follows_the_probability_model():
    r = arr(lib().jm_cabac_range_lps(), 256, ctypes.c_uint8, np.int64).reshape(64, 4)
    assert (r[63] == 2).all()
    for s in range(63):
        p = 0.5 * ALPHA ** s
        for q in range(4):
            model = p * (288 + 64 * q)
            assert abs(r[s, q] - model) <= max(2.0, 0.06 * model) or (s < 3 and q == 0 and r[s, q] == 128), (s, q, r[s, q], model)
        assert (np.diff(r[s]) > 0).all()                      # larger range -> larger LPS sub-range
    assert (np.diff(r[:63, 3]) <= 0).all()                    # more skewed state -> smaller LPS sub-range


def test_trans_lps_follows_the_probability_model():
    t = arr(lib().jm_cabac_trans_lps(), 64, ctypes.c_uint8, np.int64)
    assert t[0] == 0 and t[63] == 63
    for s in range(1, 63):
        p = ALPHA * 0.5 * ALPHA ** s + (1 - ALPHA)
        model = math.log(p / 0.5) / math.log(ALPHA)
        assert abs(t[s] - model) <= 1.0, (s, t[s], model)
        assert t[s] < s


def test_init_tables_cover_the_coded_contexts():
    h = lib()
    used_i = list(range(0, 11)) + list(range(60, 70)) + list(range(73, 105)) + list(range(105, 276)) + list(range(399, 436))
    used_p = used_i + list(range(11, 24)) + list(range(40, 54))
    for slice_i, used in ((1, used_i), (0, used_p)):
        t = arr(h.jm_cabac_init_table(slice_i), 920, ctypes.c_int8, np.int64).reshape(460, 2)
        missing = [c for c in used if t[c, 0] == 0 and t[c, 1] == 0]
        assert not missing, (slice_i, missing)
        assert (np.abs(t[:, 0]) <= 50).all() and (t[:, 1] >= -30).all() and (t[:, 1] <= 127).all()
        assert (t[276] == 0).all()                            # end_of_slice_flag: not context coded
    ti = arr(h.jm_cabac_init_table(1), 920, ctypes.c_int8, np.int64).reshape(460, 2)
    tp = arr(h.jm_cabac_init_table(0), 920, ctypes.c_int8, np.int64).reshape(460, 2)
    assert (ti[:11] == tp[:11]).all() and (ti[60:70] == tp[60:70]).all()   # shared by both tables

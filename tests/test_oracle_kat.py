"""Known-answer tests pinning the oracle to ITU-T H.264 normative arithmetic and to the JM
tables it restates (SURVEY.md §4 "Known-answer").  CPU only."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib
from jmpaths import PKG

L = oracle_lib.lib()


def arr(a, dt=np.int32):
    return np.ascontiguousarray(a, dt)


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# ---- Init_Motion_Search_Module: spiral + mvbits ----------------------------------------
def test_spiral_order_and_coverage():
    R = 16
    n = (2 * R + 1) ** 2
    sx, sy = np.zeros(n, np.int32), np.zeros(n, np.int32)
    L.jmo_spiral(R, ptr(sx), ptr(sy))
    first9 = list(zip(sx[:9], sy[:9]))
    assert first9 == [(0, 0), (0, -1), (0, 1), (-1, -1), (1, -1), (-1, 0), (1, 0), (-1, 1), (1, 1)]
    assert len(set(zip(sx.tolist(), sy.tolist()))) == n
    # spiral prefixes are squares: entries [0, (2r+1)^2) cover exactly |x|,|y| <= r
    for r in range(R + 1):
        m = (2 * r + 1) ** 2
        assert np.max(np.maximum(np.abs(sx[:m]), np.abs(sy[:m]))) == r


def se_len(v):
    k = 2 * v - 1 if v > 0 else -2 * v
    return 2 * int(np.floor(np.log2(k + 1))) + 1


@pytest.mark.parametrize("v", list(range(-300, 301, 7)) + [0, 1, -1, 2, 3, 4, 1023, -1024])
def test_mvbits_is_se_length(v):
    assert L.jmo_mvbits(v) == se_len(v)


# ---- transforms, SATD, quant ---------------------------------------------------------------
def test_forward_constant_block_is_dc_only():
    for c in (-255, -3, 0, 7, 255):
        out = np.zeros(16, np.int32)
        L.jmo_forward4x4(ptr(arr([c] * 16)), ptr(out))
        assert out[0] == 16 * c and not out[1:].any()


def test_inverse_dc_only_is_flat():
    out = np.zeros(16, np.int32)
    L.jmo_inverse4x4(ptr(arr([640] + [0] * 15)), ptr(out))
    assert (out == 640).all()


def test_inverse_known_row():
    # d = [d0,d1,d2,d3] on the first row only: e0=d0+d2, e1=d0-d2, e2=(d1>>1)-d3, e3=d1+(d3>>1)
    d = np.zeros(16, np.int32)
    d[:4] = [64, 32, -16, 8]
    out = np.zeros(16, np.int32)
    L.jmo_inverse4x4(ptr(d), ptr(out))
    e0, e1, e2, e3 = 64 - 16, 64 + 16, (32 >> 1) - 8, 32 + (8 >> 1)
    row = [e0 + e3, e1 + e2, e1 - e2, e0 - e3]
    for y in range(4):
        assert list(out[4 * y:4 * y + 4]) == row   # columns see only their DC term


def test_satd_delta():
    for a in (1, -5, 200):
        d = arr([a] + [0] * 15)
        assert L.jmo_satd4x4(ptr(d), 1) == 8 * abs(a)     # 16 |a| / 2
        assert L.jmo_satd4x4(ptr(d), 0) == abs(a)


def test_satd_sum_is_even_so_rounding_is_moot():
    rng = np.random.default_rng(0)
    for _ in range(200):
        d = arr(rng.integers(-255, 256, 16))
        assert L.jmo_satd4x4(ptr(d), 1) * 2 in range(0, 1 << 20)


def test_tq_zero_residual_and_recon_is_pred():
    pred = np.full((3, 16), 77, np.uint8)
    lev, rec, cc, nz = oracle_lib.tq4x4(np.zeros((3, 16), np.int16), pred, 28, 0)
    assert not lev.any() and (rec == 77).all() and not nz.any() and not cc.any()


def test_tq_dc_quant_known_answer():
    # residual constant 10 -> DC coefficient 160; QP 28 inter: qp_per 4, qp_rem 4,
    # level = (160*8192 + (1<<19)/6) >> 19 = 2
    lev, rec, cc, nz = oracle_lib.tq4x4(np.full((1, 16), 10, np.int16), np.full((1, 16), 100, np.uint8), 28, 0)
    assert lev[0, 0] == 2 and not lev[0, 1:].any() and nz[0] == 1
    assert cc[0] == 999999                      # |level| > 1 -> MAX_VALUE (never discarded)
    # dequant 2*16<<4 = 512; inverse flat 512 -> (512+32)>>6 = 8 -> recon 108
    assert (rec == 108).all()


def test_tq_round_trip_error_bounded_by_step():
    rng = np.random.default_rng(1)
    n = 500
    resid = rng.integers(-60, 61, (n, 16)).astype(np.int16)
    pred = rng.integers(60, 196, (n, 16)).astype(np.uint8)
    for qp in (0, 12, 24):
        _, rec, _, _ = oracle_lib.tq4x4(resid, pred, qp, 1)
        err = np.abs(rec.astype(int) - (pred.astype(int) + resid))
        qstep = 0.625 * 2 ** (qp / 6)
        assert err.max() <= max(2, 2 * qstep)


def test_qp_tables():
    assert [L.jmo_qp2quant(q) for q in (0, 12, 28, 51)] == [1, 1, 6, 91]
    assert [L.jmo_qp_scale_cr(q) for q in (0, 29, 30, 34, 39, 45, 51)] == [0, 29, 29, 32, 35, 38, 39]


# ---- 8.4.2.2.1 luma interpolation ----------------------------------------------------------
def qpel(plane, X, Y):
    h, w = plane.shape
    return L.jmo_luma_qpel_sample(ptr(plane), w, h, w, X, Y)


def test_interp_constant_plane():
    p = np.full((12, 12), 93, np.uint8)
    for X in range(-16, 60, 3):
        for Y in range(-16, 60, 5):
            assert qpel(p, X, Y) == 93


def test_interp_step_edge_half_pel():
    p = np.zeros((8, 16), np.uint8)
    p[:, 8:] = 255
    # b between x=7 and x=8: taps E..J = x 5..10 = 0,0,0,255,255,255
    b1 = 0 - 0 + 0 + 20 * 255 - 5 * 255 + 255
    assert qpel(p, 4 * 7 + 2, 4 * 3) == min(255, (b1 + 16) >> 5)
    # b between x=6 and x=7: taps 4..9 = 0,0,0,0,255,255 -> (-5*255+255+16)>>5 < 0 -> 0
    assert qpel(p, 4 * 6 + 2, 4 * 3) == 0
    # quarter a = (G + b + 1) >> 1 at x=7
    assert qpel(p, 4 * 7 + 1, 4 * 3) == (0 + min(255, (b1 + 16) >> 5) + 1) >> 1
    # vertical half-pel on a horizontal-only edge equals the column value
    assert qpel(p, 4 * 9, 4 * 3 + 2) == 255


def test_interp_outside_picture_clamps_like_edge_extension():
    rng = np.random.default_rng(2)
    p = rng.integers(0, 256, (10, 10)).astype(np.uint8)
    big = np.pad(p, 20, mode="edge")
    for X in range(-40, 80, 7):
        for Y in range(-40, 80, 9):
            assert qpel(p, X, Y) == qpel(big, X + 80, Y + 80)


# ---- 8.4.1.3 median MV prediction ----------------------------------------------------------
def mvp(a, b, c, ref=0, bsx=16, bsy=16, bx=0, by=0):
    out = np.zeros(2, np.int32)
    args = []
    for n in (a, b, c):
        av, r, x, y = n
        args += [av, r, x, y]
    L.jmo_mvp_median(*args, ref, bsx, bsy, bx, by, ptr(out))
    return tuple(out)


def test_mvp_median():
    assert mvp((1, 0, 4, -8), (1, 0, 12, 2), (1, 0, -6, 5)) == (4, 2)


def test_mvp_single_matching_reference():
    assert mvp((1, 1, 4, -8), (1, 0, 12, 2), (1, 1, -6, 5)) == (12, 2)


def test_mvp_only_left_available():
    assert mvp((1, 0, 7, 3), (0, -1, 0, 0), (0, -1, 0, 0)) == (7, 3)


def test_mvp_directional_16x8_and_8x16():
    A, B, C = (1, 0, 1, 1), (1, 0, 2, 2), (1, 0, 3, 3)
    assert mvp(A, B, C, bsx=16, bsy=8, by=0) == (2, 2)      # upper 16x8 -> B
    assert mvp(A, B, C, bsx=16, bsy=8, by=2) == (1, 1)      # lower 16x8 -> A
    assert mvp(A, B, C, bsx=8, bsy=16, bx=0) == (1, 1)      # left 8x16 -> A
    assert mvp(A, B, C, bsx=8, bsy=16, bx=2) == (3, 3)      # right 8x16 -> C


def test_mvp_intra_neighbours_count_as_ref_minus1():
    assert mvp((1, -1, 0, 0), (1, -1, 0, 0), (1, 0, 9, -9)) == (9, -9)


# ---- CAVLC tables (product writer and oracle decoder): prefix-free, spec codewords --------
def c_table(src, name):
    m = re.search(r"%s\[[^=]*=\s*(\{.*?\});" % name, src, re.S)
    return eval(m.group(1).replace("{", "[").replace("}", "]"))


@pytest.mark.parametrize("path", [os.path.join(PKG, "host", "bitstream.c"),
                                  os.path.join(os.path.dirname(PKG), "oracle", "decoder.c")])
def test_cavlc_tables_prefix_free(path):
    src = open(path).read()
    L_, C_ = c_table(src, "ct_len"), c_table(src, "ct_code")
    tables = []
    for t in range(3):
        tables.append([(C_[t][a][c], L_[t][a][c]) for a in range(4) for c in range(17) if a <= c])
    Ld, Cd = c_table(src, "ctdc_len"), c_table(src, "ctdc_code")
    tables.append([(Cd[a][c], Ld[a][c]) for a in range(4) for c in range(5) if a <= c])
    tzl, tzc = c_table(src, "tz_len"), c_table(src, "tz_code")
    tables += [list(zip(tzc[i], tzl[i])) for i in range(15)]
    rbl, rbc = c_table(src, "rb_len"), c_table(src, "rb_code")
    tables += [list(zip(rbc[i], rbl[i])) for i in range(7)]
    for tab in tables:
        words = [format(c, "0%db" % l) for c, l in tab if l > 0]
        assert len(set(words)) == len(words)
        for a in words:
            for b in words:
                assert a == b or not b.startswith(a)
        assert sum(2.0 ** -len(w) for w in words) <= 1.0
    # spot-check spec codewords (Table 9-5, 0 <= nC < 2)
    assert (C_[0][0][0], L_[0][0][0]) == (1, 1)          # "1"
    assert (C_[0][1][1], L_[0][1][1]) == (1, 2)          # "01"
    assert (C_[0][0][1], L_[0][0][1]) == (5, 6)          # "000101"
    assert (C_[0][3][3], L_[0][3][3]) == (3, 5)          # "00011"


# ---- 8x8 transform (High profile) -------------------------------------------
def hadamard8():
    h = np.array([[1]])
    while h.shape[0] < 8:
        h = np.block([[h, h], [h, -h]])
    return h


def test_satd8x8_is_matrix_hadamard():
    rng = np.random.default_rng(8)
    H = hadamard8()
    for _ in range(50):
        d = rng.integers(-255, 256, (8, 8))
        want = (int(np.abs(H @ d @ H.T).sum()) + 2) >> 2
        assert L.jmo_satd8x8(ptr(arr(d.reshape(-1))), 1) == want
        assert L.jmo_satd8x8(ptr(arr(d.reshape(-1))), 0) == int(np.abs(d).sum())


def test_forward8x8_constant_block_is_dc_only():
    for c in (-255, -1, 0, 9, 255):
        out = np.zeros(64, np.int32)
        L.jmo_forward8x8(ptr(arr([c] * 64)), ptr(out))
        assert out[0] == 64 * c and not out[1:].any()


def test_inverse8x8_dc_only_is_flat():
    out = np.zeros(64, np.int32)
    L.jmo_inverse8x8(ptr(arr([64 * 7] + [0] * 63)), ptr(out))
    assert (out == 64 * 7).all()


def inv8_py(v):
    """8.5.13.2 one-dimensional inverse, written from the spec equations."""
    d = list(v)
    a = [0] * 8
    b = [0] * 8
    a[0] = d[0] + d[4]; a[4] = d[0] - d[4]; a[2] = (d[2] >> 1) - d[6]; a[6] = d[2] + (d[6] >> 1)
    b[0] = a[0] + a[6]; b[2] = a[4] + a[2]; b[4] = a[4] - a[2]; b[6] = a[0] - a[6]
    a[1] = -d[3] + d[5] - d[7] - (d[7] >> 1); a[3] = d[1] + d[7] - d[3] - (d[3] >> 1)
    a[5] = -d[1] + d[7] + d[5] + (d[5] >> 1); a[7] = d[3] + d[5] + d[1] + (d[1] >> 1)
    b[1] = a[1] + (a[7] >> 2); b[7] = a[7] - (a[1] >> 2); b[3] = a[3] + (a[5] >> 2); b[5] = (a[3] >> 2) - a[5]
    return [b[0] + b[7], b[2] + b[5], b[4] + b[3], b[6] + b[1], b[6] - b[1], b[4] - b[3], b[2] - b[5], b[0] - b[7]]


def test_inverse8x8_matches_spec_equations():
    rng = np.random.default_rng(9)
    for _ in range(30):
        c = rng.integers(-4096, 4096, (8, 8))
        t = np.array([inv8_py(r) for r in c])
        want = np.array([inv8_py(col) for col in t.T]).T
        out = np.zeros(64, np.int32)
        L.jmo_inverse8x8(ptr(arr(c.reshape(-1))), ptr(out))
        assert (out.reshape(8, 8) == want).all()


def test_tq8x8_zero_residual_and_round_trip_bounded():
    rng = np.random.default_rng(10)
    pred = rng.integers(0, 256, (6, 64)).astype(np.uint8)
    lev, rec, cc, nz = oracle_lib.tq8x8(np.zeros((6, 64), np.int16), pred, 28, 1)
    assert not lev.any() and (rec == pred).all() and not nz.any() and not cc.any()
    org = rng.integers(0, 256, (40, 64))
    pred = rng.integers(0, 256, (40, 64)).astype(np.uint8)
    for qp in (0, 6, 12):
        lev, rec, cc, nz = oracle_lib.tq8x8((org - pred).astype(np.int16), pred, qp, 1)
        # quantiser step 0.625 * 2^(qp/6); the 8x8 basis error stays within a few steps
        assert np.abs(rec.astype(int) - org).max() <= 2 + (1 << (qp // 6)), qp


def test_tq8x8_coeff_cost_counts_runs():
    # a single +-1 level at scan position k costs COEFF_COST8x8[k] (3,3,3,3,2x8,1x12,0...)
    want = [3] * 4 + [2] * 8 + [1] * 12 + [0] * 40
    scan = []
    for s in range(15):
        xs = range(min(s, 7), -1, -1) if s & 1 else range(max(0, s - 7), min(s, 7) + 1)
        scan += [(s - x) * 8 + x for x in xs if 0 <= s - x < 8]
    assert len(scan) == 64 and len(set(scan)) == 64
    lev, rec, cc, nz = oracle_lib.tq8x8(np.zeros((1, 64), np.int16), np.full((1, 64), 128, np.uint8), 0, 0)
    assert cc[0] == 0
    out = np.zeros(64, np.int32)
    for k in (0, 3, 4, 11, 12, 23, 24, 63):
        # craft a residual whose transform has (mostly) one coefficient: inverse of a unit level
        c = np.zeros(64, np.int32)
        c[scan[k]] = 64
        L.jmo_inverse8x8(ptr(c), ptr(out))
        r = ((out + 32) >> 6).astype(np.int16)
        lev, _, cc, _ = oracle_lib.tq8x8(r.reshape(1, 64), np.full((1, 64), 128, np.uint8), 24, 0)
        nzk = np.flatnonzero(lev[0])
        if len(nzk) == 1 and abs(lev[0][nzk[0]]) == 1:
            assert cc[0] == want[nzk[0]]


def test_intra8x8_dc_and_vertical_known_answers():
    nb = np.zeros(25, np.int32)
    nb[0] = 100
    nb[1:17] = np.arange(16) * 10        # top row p[0..15,-1]
    nb[17:25] = 50                       # left column
    pred = np.zeros((9, 64), np.uint8)
    ok = L.jmo_intra8x8_pred(ptr(nb), 1 | 2 | 4 | 8, ptr(pred))
    assert ok == 0x1FF
    # filtered top row: p'[0] = (100 + 0 + 10 + 2) >> 2, p'[x] = 10x for a linear ramp inside
    T = [(100 + 2 * 0 + 10 + 2) >> 2] + [10 * x for x in range(1, 8)]
    assert list(pred[0][:8]) == T and all(list(pred[0][8 * y:8 * y + 8]) == T for y in range(8))
    L_ = [(100 + 2 * 50 + 50 + 2) >> 2] + [50] * 7
    assert (pred[2] == (sum(T) + sum(L_) + 8) >> 4).all()
    assert all((pred[1][8 * y:8 * y + 8] == L_[y]).all() for y in range(8))
    ok = L.jmo_intra8x8_pred(ptr(nb), 0, ptr(pred))
    assert ok == 1 << 2 and (pred[2] == 128).all()

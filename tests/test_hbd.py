"""High 10 sample path (config 5, SURVEY.md §7 hard part 7): the per-block
BlockMotionSearch, SetupFastFullPelSearch's SAD table and dct_luma / dct_luma8x8 on 16-bit
samples (include/jmhip.h jmh_*_u16; oracle/hbd.c).

CPU tests pin the 10-bit oracle: at bit depth 8 on 16-bit samples it must equal the 8-bit
oracle exactly (independent code paths), and its quarter-pel samples and transform are checked
against a small numpy restatement of H.264 8.4.2.2.1 / 8.5.12 at 10 bits, extremes 0 / 1023
included.  GPU tests compare the device seams with the oracle bit for bit.  JM parity itself is
unpinned (no JM source or 10-bit fixtures exist in /root/reference).
"""
import numpy as np
import pytest

import oracle_lib
from jmpaths import load_jmhip
from test_jm_surface import block_requests

jmhip = load_jmhip()


def pic10(w, h, seed, i, bd=10):
    """16-bit luma: the synthetic 8-bit texture scaled to bd bits plus noise, clipped."""
    y = jmhip.synth_frame(w, h, seed, i)[0].astype(np.int32) << (bd - 8)
    rng = np.random.default_rng(1000 * seed + i)
    y += rng.integers(-(1 << (bd - 8)) - 1, (1 << (bd - 8)) + 2, y.shape)
    return np.clip(y, 0, (1 << bd) - 1).astype(np.uint16)


def extreme_pic(w, h, seed, bd=10):
    """0 / max stripes and checkers: the 6-tap overshoots both ways (Clip1Y at 0 and 2^bd - 1)."""
    rng = np.random.default_rng(seed)
    m = (1 << bd) - 1
    yy, xx = np.mgrid[0:h, 0:w]
    y = np.where(((xx // int(rng.integers(1, 4))) + (yy // int(rng.integers(1, 4)))) % 2 == 0, m, 0)
    return y.astype(np.uint16)


# ---------------- numpy restatement (independent of both C paths) ----------------
def tap6(a, b, c, d, e, f):
    return a - 5 * b + 20 * c + 20 * d - 5 * e + f


def np_qpel(ref, X, Y, bd):
    """H.264 8.4.2.2.1 luma sample at quarter-pel (X, Y), coordinates clamped, Clip1Y at bd."""
    h, w = ref.shape
    mx = (1 << bd) - 1
    P = lambda x, y: int(ref[min(max(y, 0), h - 1), min(max(x, 0), w - 1)])
    clip = lambda v: min(max(v, 0), mx)
    x, y, fx, fy = X >> 2, Y >> 2, X & 3, Y & 3
    hb1 = lambda x, y: tap6(*(P(x + k, y) for k in range(-2, 4)))
    vh1 = lambda x, y: tap6(*(P(x, y + k) for k in range(-2, 4)))
    G = P(x, y)
    b, hh = clip((hb1(x, y) + 16) >> 5), clip((vh1(x, y) + 16) >> 5)
    s, m = clip((hb1(x, y + 1) + 16) >> 5), clip((vh1(x + 1, y) + 16) >> 5)
    j = clip((tap6(*(vh1(x + k, y) for k in range(-2, 4))) + 512) >> 10)
    return [G, (G + b + 1) >> 1, b, (P(x + 1, y) + b + 1) >> 1, (G + hh + 1) >> 1, (b + hh + 1) >> 1, (b + j + 1) >> 1,
            (b + m + 1) >> 1, hh, (hh + j + 1) >> 1, j, (j + m + 1) >> 1, (P(x, y + 1) + hh + 1) >> 1, (hh + s + 1) >> 1,
            (j + s + 1) >> 1, (m + s + 1) >> 1][fy * 4 + fx]


QC = [[13107, 5243, 8066], [11916, 4660, 7490], [10082, 4194, 6554], [9362, 3647, 5825], [8192, 3355, 5243], [7282, 2893, 4559]]
DQ = [[10, 16, 13], [11, 18, 14], [13, 20, 16], [14, 23, 18], [16, 25, 20], [18, 29, 23]]
SCAN = [0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15]
COST = [3, 2, 2, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0]


def np_dct_luma(resid, pred, qp, intra, bd):
    """dct_luma [J] at qp + 6 (bd - 8) (8.5.12 inverse; JM 8.6 or JM >= 10 rounding offsets)."""
    C = np.array([[1, 1, 1, 1], [2, 1, -1, -2], [1, -1, -1, 1], [1, -2, 2, -1]], np.int64)
    m = C @ resid.reshape(4, 4).astype(np.int64) @ C.T
    qpb = qp + 6 * (bd - 8)
    per, rem, qb = qpb // 6, qpb % 6, 15 + qpb // 6
    # intra: the rounding selector (0 / 1 JM 8.6 / 6 and / 3; 2 + o JM >= 10 offset o at OffsetBits 11)
    const = (intra - 2) << (qb - 11) if intra >= 2 else (1 << qb) // 3 if intra else (1 << qb) // 6
    lev = np.zeros(16, np.int64)
    dq = np.zeros((4, 4), np.int64)
    cost, run = 0, -1
    for k, pos in enumerate(SCAN):
        yy, xx = divmod(pos, 4)
        cls = 0 if (xx | yy) % 2 == 0 else (1 if (xx & yy) % 2 == 1 else 2)
        run += 1
        level = (abs(int(m[yy, xx])) * QC[rem][cls] + const) >> qb
        if level:
            cost += 999999 if level > 1 else COST[run]
            run = -1
            s = -1 if m[yy, xx] < 0 else 1
            lev[k] = s * level
            dq[yy, xx] = s * ((level * DQ[rem][cls]) << per)

    def inv1(d):
        e0, e1, e2, e3 = d[0] + d[2], d[0] - d[2], (d[1] >> 1) - d[3], d[1] + (d[3] >> 1)
        return np.array([e0 + e3, e1 + e2, e1 - e2, e0 - e3])
    t = np.array([inv1(r) for r in dq])
    r = np.array([inv1(c) for c in t.T]).T
    rec = np.clip((r.reshape(16) + (pred.astype(np.int64) << 6) + 32) >> 6, 0, (1 << bd) - 1)
    return lev, rec, cost


# ---------------- CPU: the oracle pinned ----------------
@pytest.mark.parametrize("intra", [0, 1])
def test_oracle_hbd_tq_at_8_bits_equals_8bit_oracle(intra):
    rng = np.random.default_rng(5 + intra)
    for el, f8 in ((16, oracle_lib.tq4x4), (64, oracle_lib.tq8x8)):
        resid = rng.integers(-255, 256, (200, el)).astype(np.int16)
        resid[:8] = np.where(rng.random((8, el)) < 0.5, 255, -255)
        pred = rng.integers(0, 256, (200, el)).astype(np.uint8)
        for qp in range(0, 52, 3):
            a = f8(resid, pred, qp, intra)
            b = oracle_lib.tq_u16(resid, pred.astype(np.uint16), qp, intra, 8)
            for x, y in zip(a, b):
                assert np.array_equal(np.asarray(x, np.int64), np.asarray(y, np.int64)), (el, qp)


@pytest.mark.parametrize("bd", [9, 10])
def test_oracle_hbd_tq4x4_matches_numpy(bd):
    rng = np.random.default_rng(bd)
    mx = (1 << bd) - 1
    resid = rng.integers(-mx, mx + 1, (64, 16)).astype(np.int16)
    resid[:4] = np.where(rng.random((4, 16)) < 0.5, mx, -mx)
    pred = rng.integers(0, mx + 1, (64, 16)).astype(np.uint16)
    for qp in (0, 7, 20, 28, 37, 51):
        for intra in (0, 1):
            lev, rec, cc, nz = oracle_lib.tq_u16(resid, pred, qp, intra, bd)
            for i in range(0, 64, 7):
                l2, r2, c2 = np_dct_luma(resid[i], pred[i], qp, intra, bd)
                assert np.array_equal(lev[i], l2) and np.array_equal(rec[i], r2) and cc[i] == c2, (qp, intra, i)


def test_oracle_hbd_qpel_matches_numpy_with_clipping():
    w, h = 64, 48
    for ref, bd in ((extreme_pic(w, h, 3), 10), (pic10(w, h, 2, 0), 10), (extreme_pic(w, h, 4, 9), 9)):
        o = oracle_lib.OracleHbd(w, h, 4)
        o.pictures(ref, ref, bd)
        rng = np.random.default_rng(bd)
        vals = []
        for _ in range(400):
            X, Y = int(rng.integers(-12, 4 * w + 12)), int(rng.integers(-12, 4 * h + 12))
            v = o.qpel(X, Y)
            assert v == np_qpel(ref, X, Y, bd), (X, Y)
            vals.append(v)
        assert max(vals) <= (1 << bd) - 1 and min(vals) >= 0


def test_oracle_hbd_search_at_8_bits_equals_8bit_oracle():
    w, h, sr = 96, 64, 8
    pics = [jmhip.synth_frame(w, h, 6, i)[0] for i in range(2)]
    for had in (1, 0):
        o8 = oracle_lib.OracleEncoder(w, h, search_range=sr, use_hadamard=had)
        o8.search_pictures(pics[1], pics[0])
        o16 = oracle_lib.OracleHbd(w, h, sr, use_hadamard=had)
        o16.pictures(pics[1].astype(np.uint16), pics[0].astype(np.uint16), 8)
        reqs = block_requests(w, h, sr, 60, 3 + had)
        for i, (a, b) in enumerate(zip(o8.block_motion_search(reqs), o16.block_motion_search(reqs))):
            assert bytes(a) == bytes(b), (i, list(a.mv), a.min_mcost, list(b.mv), b.min_mcost)
        mbxy = np.array([[0, 0], [5, 3], [2, 1]], np.int32)
        cen = np.array([[0, 0], [-8, 8], [3, -2]], np.int32)
        o8.load_current(*jmhip.synth_frame(w, h, 6, 1))
        o8.set_reference(*jmhip.synth_frame(w, h, 6, 0))
        assert np.array_equal(o8.sad_table(mbxy, cen), o16.sad_table(mbxy, cen))


# ---------------- GPU: device seams == oracle ----------------
@pytest.mark.gpu
@pytest.mark.parametrize("bd", [10, 9, 8])
def test_gpu_hbd_tq_all_qp(bd):
    rng = np.random.default_rng(40 + bd)
    mx = (1 << bd) - 1
    g = jmhip.Encoder(64, 64, search_range=4)
    for el in (16, 64):
        resid = rng.integers(-mx, mx + 1, (96, el)).astype(np.int16)
        resid[:16] = np.where(rng.random((16, el)) < 0.5, mx, -mx)         # extremes: +-1023
        resid[16:20] = 0
        pred = rng.integers(0, mx + 1, (96, el)).astype(np.uint16)
        pred[:8] = np.where(rng.random((8, el)) < 0.5, mx, 0)
        for qp in range(52):
            for intra in (0, 1):
                a = g.tq_u16(resid, pred, qp, intra, bd)
                b = oracle_lib.tq_u16(resid, pred, qp, intra, bd)
                for x, y in zip(a, b):
                    assert np.array_equal(x, y), (el, qp, intra)
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,sr,had,bd", [(176, 144, 16, 1, 10), (176, 144, 16, 0, 10), (352, 288, 32, 1, 10), (176, 144, 8, 1, 9)])
def test_gpu_hbd_block_motion_search(w, h, sr, had, bd):
    """jmh_block_motion_search_u16 == the 10-bit oracle on random requests (all block types,
    FFS and full search, edge MBs), QCIF and CIF; costs above 16 bits occur."""
    cur, ref = pic10(w, h, 7, 1, bd), pic10(w, h, 7, 0, bd)
    if w >= 352:   # a saturated current picture: 16x16 costs above 16 bits (the 19-bit key path)
        cur = np.full_like(cur, (1 << bd) - 1)
    g = jmhip.Encoder(w, h, search_range=sr, use_hadamard=had)
    o = oracle_lib.OracleHbd(w, h, sr, use_hadamard=had)
    g.search_pictures_u16(cur, ref, bd)
    o.pictures(cur, ref, bd)
    reqs = block_requests(w, h, sr, 200, 21 + had + bd)
    gr, orr = g.block_motion_search_u16(reqs), o.block_motion_search(reqs)
    for i, (a, b) in enumerate(zip(gr, orr)):
        assert bytes(a) == bytes(b), (i, list(a.mv), a.min_mcost, list(b.mv), b.min_mcost)
    assert max(r.fullpel_cost for r in orr) > 65535 or w < 352   # CIF exercises 19-bit costs
    g.close()


@pytest.mark.gpu
def test_gpu_hbd_extremes_and_sad_table():
    """Saturated 0 / 1023 pictures (the 6-tap overshoots both ways) through the per-block search
    and the SAD table (v_sad_u16)."""
    w, h, sr = 96, 64, 8
    cur, ref = extreme_pic(w, h, 11), extreme_pic(w, h, 12)
    g = jmhip.Encoder(w, h, search_range=sr)
    o = oracle_lib.OracleHbd(w, h, sr)
    g.search_pictures_u16(cur, ref, 10)
    o.pictures(cur, ref, 10)
    reqs = block_requests(w, h, sr, 120, 5)
    for a, b in zip(g.block_motion_search_u16(reqs), o.block_motion_search(reqs)):
        assert bytes(a) == bytes(b)
    mbxy = np.array([[x, y] for y in range(h // 16) for x in range(w // 16)], np.int32)
    cen = np.random.default_rng(3).integers(-sr, sr + 1, mbxy.shape).astype(np.int32)
    assert np.array_equal(g.sad_table_u16(mbxy, cen), o.sad_table(mbxy, cen))
    cur, ref = pic10(w, h, 8, 1), pic10(w, h, 8, 0)
    g.search_pictures_u16(cur, ref, 10)
    o.pictures(cur, ref, 10)
    assert np.array_equal(g.sad_table_u16(mbxy, cen), o.sad_table(mbxy, cen))
    g.close()


@pytest.mark.gpu
def test_gpu_hbd_at_8_bits_equals_8bit_seams():
    """The 16-bit seams at bit depth 8 give exactly the 8-bit seams' results on the device."""
    w, h, sr = 176, 144, 16
    pics = [jmhip.synth_frame(w, h, 4, i)[0] for i in range(2)]
    g = jmhip.Encoder(w, h, search_range=sr)
    g.search_pictures(pics[1], pics[0])
    g.search_pictures_u16(pics[1].astype(np.uint16), pics[0].astype(np.uint16), 8)
    reqs = block_requests(w, h, sr, 150, 9)
    for a, b in zip(g.block_motion_search(reqs), g.block_motion_search_u16(reqs)):
        assert bytes(a) == bytes(b)
    g.close()

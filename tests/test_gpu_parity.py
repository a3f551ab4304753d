"""GPU parity: the MI355X path (through the C ABI) must equal the oracle bit for bit.

Covers every §8 row the GPU implements: a1 interpolation (qpel planes), a2 FFS SAD table,
a3-a8 motion search (through whole-picture results), a9 mode decision, a10-a14 TQ + recon,
and the lencod bitstream end to end.  Sizes are chosen so the oracle finishes in seconds;
the 1080p cases use the size-independent closed-loop property (decoder output == recon).
"""
import ctypes
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib
from jmpaths import JMDEC, LENCOD, LENCOD_CPU, ensure_built, load_jmhip

jmhip = load_jmhip()
pytestmark = pytest.mark.gpu

FIELDS = [n for n in jmhip.MB_RESULT_DTYPE.names if n not in ("pad0", "reserved")]


def first_mismatch(a, b, mbw):
    for i in range(len(a)):
        for f in FIELDS:
            if not np.array_equal(a[i][f], b[i][f]):
                return f"MB {i} (x={i % mbw}, y={i // mbw}) field '{f}': gpu={a[i][f]!r} oracle={b[i][f]!r}"
    return None


def assert_same(gres, grec, ores, orec, mbw):
    msg = first_mismatch(gres, ores, mbw)
    assert msg is None, msg
    for k, (g, o) in enumerate(zip(grec, orec)):
        if not np.array_equal(g, o):
            yy, xx = np.argwhere(g != o)[0]
            pytest.fail(f"recon plane {k} differs first at ({xx},{yy}): gpu={g[yy, xx]} oracle={o[yy, xx]}")


def rand_picture(rng, w, h, smooth=True):
    y = rng.integers(0, 256, (h, w), dtype=np.uint8)
    if smooth:   # mixture of texture and flat areas (exercises ties and intra modes)
        base = np.cumsum(rng.integers(-3, 4, (h, w)), axis=1).astype(np.int32)
        y = np.clip(128 + base + rng.integers(-2, 3, (h, w)), 0, 255).astype(np.uint8)
        y[: h // 3, : w // 3] = 77
    u = rng.integers(0, 256, (h // 2, w // 2), dtype=np.uint8)
    v = rng.integers(0, 256, (h // 2, w // 2), dtype=np.uint8)
    return y, u, v


@pytest.fixture(scope="module", autouse=True)
def built():
    ensure_built()
    jmhip.load()


# ---------------- a1: quarter-pel interpolation ----------------
@pytest.mark.parametrize("w,h", [(64, 48), (176, 144)])
def test_qpel_planes(w, h):
    rng = np.random.default_rng(1)
    ref = rand_picture(rng, w, h, smooth=False)
    g = jmhip.Encoder(w, h, search_range=8)
    o = oracle_lib.OracleEncoder(w, h, search_range=8)
    g.set_reference(*ref)
    o.set_reference(*ref)
    assert np.array_equal(g.read_qpel(), o.read_qpel())


# ---------------- a11: 4x4 TQ + recon ----------------
@pytest.mark.parametrize("intra", [0, 1])
def test_tq4x4_all_qp(intra):
    rng = np.random.default_rng(2)
    g = jmhip.Encoder(32, 32, search_range=4)
    n = 4096
    resid = rng.integers(-255, 256, (n, 16)).astype(np.int16)
    resid[:64] = 255          # max-magnitude residuals
    resid[64:128] = -255
    resid[128:192] = 0
    pred = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    for qp in range(52):
        a = g.tq4x4(resid, pred, qp, intra)
        b = oracle_lib.tq4x4(resid, pred, qp, intra)
        for x, y in zip(a, b):
            assert np.array_equal(x, y), f"qp {qp}"


# ---------------- a12: 8x8 TQ + recon (High profile) ----------------
@pytest.mark.parametrize("intra", [0, 1])
def test_tq8x8_all_qp(intra):
    rng = np.random.default_rng(12)
    g = jmhip.Encoder(32, 32, search_range=4)
    n = 1024
    resid = rng.integers(-255, 256, (n, 64)).astype(np.int16)
    resid[:16] = 255          # max-magnitude residuals
    resid[16:32] = -255
    resid[32:48] = 0
    resid[48:64] = rng.integers(-2, 3, (16, 64))    # sparse levels: COEFF_COST8x8 runs
    pred = rng.integers(0, 256, (n, 64)).astype(np.uint8)
    for qp in range(52):
        a = g.tq8x8(resid, pred, qp, intra)
        b = oracle_lib.tq8x8(resid, pred, qp, intra)
        for x, y in zip(a, b):
            assert np.array_equal(x, y), f"qp {qp}"


# ---------------- a2: FFS SAD table ----------------
@pytest.mark.parametrize("sr", [4, 16, 32])
def test_sad_table(sr):
    rng = np.random.default_rng(3)
    w, h = 96, 64
    cur, ref = rand_picture(rng, w, h), rand_picture(rng, w, h)
    g = jmhip.Encoder(w, h, search_range=sr)
    o = oracle_lib.OracleEncoder(w, h, search_range=sr)
    g.set_reference(*ref)
    o.set_reference(*ref)
    g.load_frame(0, *cur)
    o.load_current(*cur)
    mb_xy = [(0, 0), (5, 3), (2, 1), (5, 0), (0, 3)]
    centres = [(0, 0), (sr, -sr), (-3, 2), (-sr, sr), (7, -1)]
    assert np.array_equal(g.sad_table(mb_xy, centres), o.sad_table(mb_xy, centres))


# ---------------- a3..a14: whole pictures ----------------
def encode_pair(w, h, frames, slice_types, qp, first_ref=None, **kw):
    g = jmhip.Encoder(w, h, **kw)
    o = oracle_lib.OracleEncoder(w, h, **kw)
    if first_ref is not None:
        g.set_reference(*first_ref)
        o.set_reference(*first_ref)
    for i, (pic, st) in enumerate(zip(frames, slice_types)):
        gres, grec = g.encode(*pic, st, qp)
        ores, orec = o.encode(*pic, st, qp)
        assert_same(gres, grec, ores, orec, w // 16)
        # next reference = this reconstruction (deblocking is host-side and not under test here)
        g.set_reference(*orec)
        o.set_reference(*orec)
    return True


def synth_seq(w, h, n, seed):
    return [jmhip.synth_frame(w, h, seed, i) for i in range(n)]


def test_intra_picture_qcif():
    pics = synth_seq(176, 144, 1, 3)
    encode_pair(176, 144, pics, [jmhip.JMH_I_SLICE], 28, search_range=16)


def test_ippp_qcif_sr16():
    pics = synth_seq(176, 144, 4, 1)
    encode_pair(176, 144, pics, [jmhip.JMH_I_SLICE] + [jmhip.JMH_P_SLICE] * 3, 28, search_range=16)


@pytest.mark.parametrize("kw,qp", [
    (dict(search_range=8, use_hadamard=0), 28),
    (dict(search_range=8, restrict_search_range=0), 24),
    (dict(search_range=8, restrict_search_range=1), 32),
    (dict(search_range=4, inter_search=(0, 1, 1, 1, 0, 1, 0)), 28),
    (dict(search_range=4, inter_search=(1, 0, 0, 0, 0, 0, 0)), 20),
    (dict(search_range=4), 0),
    (dict(search_range=4), 51),
    (dict(search_range=32), 28),
    (dict(search_range=8, search_mode=-1), 28),                              # FullPelBlockMotionSearch
    (dict(search_range=16, search_mode=-1, restrict_search_range=0), 30),
    (dict(search_range=8, search_mode=-1, use_hadamard=0, inter_search=(1, 1, 0, 1, 1, 0, 1)), 36),
    # EPZS (SearchMode 3, a15): predictors, thresholds, diamond refinement, temporal predictors
    (dict(search_range=16, search_mode=3), 28),
    (dict(search_range=32, search_mode=3, restrict_search_range=0), 20),
    (dict(search_range=8, search_mode=3, use_hadamard=0, inter_search=(1, 0, 1, 1, 0, 1, 1)), 36),
    (dict(search_range=4, search_mode=3, inter_search=(0, 1, 1, 1, 1, 1, 1)), 44),
    # SliceMode 1 (f4's slice structure): one MB row, ragged runs, one MB per slice
    (dict(search_range=8, slice_mbs=6), 28),
    (dict(search_range=8, slice_mbs=5), 24),
    (dict(search_range=4, slice_mbs=1), 30),
    (dict(search_range=8, search_mode=-1, slice_mbs=7), 28),
    (dict(search_range=16, search_mode=3, slice_mbs=6), 28),
    (dict(search_range=16, search_mode=3, slice_mbs=1, epzs_dual_refinement=1), 32),
])
def test_ipp_configs(kw, qp):
    pics = synth_seq(96, 64, 3, 7)
    encode_pair(96, 64, pics, [jmhip.JMH_I_SLICE, jmhip.JMH_P_SLICE, jmhip.JMH_P_SLICE], qp, **kw)


@pytest.mark.parametrize("kw,qp", [
    (dict(search_range=16), 28),
    (dict(search_range=8), 40),                                    # mostly Intra8x8 I pictures
    (dict(search_range=8, use_hadamard=0), 8),
    (dict(search_range=8), 0),
    (dict(search_range=8), 51),
    (dict(search_range=8, inter_search=(1, 1, 1, 1, 0, 0, 0)), 24),   # P8x8 with 8x8 sub-blocks only
    (dict(search_range=8, search_mode=-1, restrict_search_range=0), 33),
    (dict(search_range=8, slice_mbs=5), 28),                       # Intra8x8 neighbours across slice edges
    (dict(search_range=16, search_mode=3, slice_mbs=6), 30),
])
def test_high_profile_transform8x8(kw, qp):
    """a12 + Intra8x8 (Transform8x8Mode = 1): k_mb_intra8, TransformDecision, dct_luma8x8."""
    pics = synth_seq(96, 64, 3, 17)
    encode_pair(96, 64, pics, [jmhip.JMH_I_SLICE, jmhip.JMH_P_SLICE, jmhip.JMH_P_SLICE], qp,
                transform_8x8_mode=1, **kw)


def test_high_profile_qcif_ippp():
    pics = synth_seq(176, 144, 4, 21)
    for qp in (20, 30, 38):
        encode_pair(176, 144, pics, [jmhip.JMH_I_SLICE] + [jmhip.JMH_P_SLICE] * 3, qp, search_range=16,
                    transform_8x8_mode=1)


@pytest.mark.parametrize("qp", [16, 30])
def test_epzs_moving_sequence(qp):
    """a15: EPZS on large motion (window rings, temporal predictors from the previous picture's
    motion field, spatial memory), High profile on top; GPU == oracle bit for bit."""
    pics = moving_seq(176, 144, 5, seed=9, step=(13, -7))
    encode_pair(176, 144, pics, [jmhip.JMH_I_SLICE] + [jmhip.JMH_P_SLICE] * 4, qp, search_range=32, search_mode=3,
                transform_8x8_mode=1)


def shear_seq(w, h, n, seed):
    """Vertical bands moving in opposite directions (+30 / -30 px horizontally, +-20 vertically):
    sub-block MVPs at the band edges differ from the macroblock's 16x16 MVP by ~60 px, so EPZS
    candidates and sub-pel neighbourhoods leave k_mb_epzs's LDS window (the global-memory path)."""
    rng = np.random.default_rng(seed)
    big = rand_picture(rng, w + 64 * n + 128, h + 48 * n + 128)[0]
    pics = []
    for i in range(n):
        y = np.empty((h, w), np.uint8)
        for b0 in range(0, w, 24):
            sgn = 1 if (b0 // 24) % 2 == 0 else -1
            x0, y0 = 64 + 32 * n + sgn * 30 * i + b0, 64 + 24 * n + sgn * 20 * i
            y[:, b0:b0 + 24] = big[y0:y0 + h, x0:x0 + min(24, w - b0)]
        y = np.clip(y.astype(np.int16) + rng.integers(-4, 5, y.shape), 0, 255).astype(np.uint8)
        pics.append((np.ascontiguousarray(y), np.ascontiguousarray(y[::2, ::2] // 2 + 40), np.ascontiguousarray(255 - y[1::2, 1::2])))
    return pics


@pytest.mark.parametrize("t8", [0, 1])
def test_epzs_window_misses(t8):
    """EPZS with motion that leaves the 120x120 LDS window (opposite shears): GPU == oracle."""
    pics = shear_seq(176, 144, 4, seed=51)
    encode_pair(176, 144, pics, [jmhip.JMH_I_SLICE] + [jmhip.JMH_P_SLICE] * 3, 26, search_range=32, search_mode=3,
                transform_8x8_mode=t8)


def test_config3_width_3840_epzs():
    """Config 3 at its real width (3840, as 3840x2160 in the bench): High profile, EPZS + 8x8
    transform, SR 32, an I picture and two P pictures under large motion and with the temporal
    predictors of the previous P picture; GPU == oracle on every macroblock."""
    w, h = 3840, 256
    pics = moving_seq(w, h, 3, seed=38, step=(37, -29))
    encode_pair(w, h, pics, [jmhip.JMH_I_SLICE, jmhip.JMH_P_SLICE, jmhip.JMH_P_SLICE], 28, search_range=32, search_mode=3,
                transform_8x8_mode=1)


@pytest.mark.parametrize("slice_mbs", [240, 173])
def test_config5_slices_width_3840(slice_mbs):
    """Config 5's slice structure at its real width: SliceArgument 240 = one 3840-wide MB row per
    slice (and a ragged 173), High profile, EPZS + 8x8 transform, under large motion; GPU ==
    oracle on every macroblock (8-bit samples: the 10-bit wavefront and CABAC / RDO are not
    built)."""
    w, h = 3840, 128
    pics = moving_seq(w, h, 3, seed=40, step=(29, -23))
    encode_pair(w, h, pics, [jmhip.JMH_I_SLICE, jmhip.JMH_P_SLICE, jmhip.JMH_P_SLICE], 28, search_range=32, search_mode=3,
                transform_8x8_mode=1, slice_mbs=slice_mbs)


def test_random_content_p_frames():
    rng = np.random.default_rng(11)
    pics = [rand_picture(rng, 64, 64) for _ in range(3)]
    ref = rand_picture(rng, 64, 64, smooth=False)
    encode_pair(64, 64, pics, [jmhip.JMH_P_SLICE] * 3, 26, first_ref=ref, search_range=16)


def test_flat_frames_ties():
    flat = (np.full((48, 64), 100, np.uint8), np.full((24, 32), 128, np.uint8), np.full((24, 32), 128, np.uint8))
    encode_pair(64, 48, [flat, flat], [jmhip.JMH_P_SLICE, jmhip.JMH_P_SLICE], 28, first_ref=flat, search_range=8)


def test_saturated_frames():
    rng = np.random.default_rng(5)
    pics = []
    for _ in range(2):
        y = (rng.integers(0, 2, (48, 64)) * 255).astype(np.uint8)
        pics.append((y, np.zeros((24, 32), np.uint8), np.full((24, 32), 255, np.uint8)))
    encode_pair(64, 48, pics, [jmhip.JMH_I_SLICE, jmhip.JMH_P_SLICE], 18, search_range=8)


def test_device_resident_deblocked_reference():
    """f2: the slot path (encode_slot with the fused loop filter, set_reference_slot(-2) makes the
    deblocked picture the reference on the device) == the host-copy path (encode, read_deblocked,
    set_reference)."""
    w, h, qp, dbk = 96, 64, 30, (0, 1, -2)
    pics = synth_seq(w, h, 4, 11)
    a = jmhip.Encoder(w, h, search_range=8, slots=3)
    b = jmhip.Encoder(w, h, search_range=8)
    for i in range(3):
        a.load_frame(i, *pics[i])
    a.encode_slot(0, jmhip.JMH_I_SLICE, qp, deblock=dbk)
    for i in (1, 2):
        a.set_reference_slot(-2)
        a.encode_slot(i, jmhip.JMH_P_SLICE, qp, deblock=dbk)
    a.set_reference_slot(-2)
    ares, arec = a.encode(*pics[3], jmhip.JMH_P_SLICE, qp, deblock=dbk)
    adbk = a.deblocked()
    for i in range(3):
        b.encode(*pics[i], jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE, qp, deblock=dbk)
        b.set_reference(*b.deblocked())
    bres, brec = b.encode(*pics[3], jmhip.JMH_P_SLICE, qp, deblock=dbk)
    assert_same(ares, arec, bres, brec, w // 16)
    for x, y in zip(adbk, b.deblocked()):
        assert np.array_equal(x, y)
    a.encode_slot(1, jmhip.JMH_P_SLICE, qp)   # no loop filter: no deblocked picture to reference
    with pytest.raises(jmhip.JmhError):
        a.set_reference_slot(-2)


# ---------------- pipelined pictures (several pictures per wavefront tick) ----------------
def moving_seq(w, h, n, seed, step=(37, -29)):
    """Smooth random texture under large global motion (MVs near the window edge) plus noise."""
    rng = np.random.default_rng(seed)
    big = rand_picture(rng, w + abs(step[0]) * n + 64, h + abs(step[1]) * n + 64)[0]
    pics = []
    for i in range(n):
        x0 = 32 + (i * step[0] if step[0] >= 0 else (n - i) * -step[0])
        y0 = 32 + (i * step[1] if step[1] >= 0 else (n - i) * -step[1])
        y = big[y0:y0 + h, x0:x0 + w].copy()
        y = np.clip(y.astype(np.int16) + rng.integers(-6, 7, y.shape), 0, 255).astype(np.uint8)
        u = np.ascontiguousarray(y[::2, ::2] // 2 + 40)
        v = np.ascontiguousarray(255 - y[1::2, 1::2])
        pics.append((np.ascontiguousarray(y), u, v))
    return pics


def run_chain(enc, pics, qp, dbk, pipelined):
    """IPPP chain, each P referencing the previous picture's device deblocking."""
    out, pending = [], 0
    for i, pic in enumerate(pics):
        st = jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE
        if i:
            enc.set_reference_slot(-2)
        if pipelined:
            if pending == enc.depth:
                out.append(enc.pop() + (enc.deblocked(),))
                pending -= 1
            enc.push(*pic, st, qp, deblock=dbk)
            pending += 1
        else:
            out.append(enc.encode(*pic, st, qp, deblock=dbk) + (enc.deblocked(),))
    for _ in range(pending):
        out.append(enc.pop() + (enc.deblocked(),))
    return out


# SearchRange > 32 (EPZS only, VERDICT r5 missing #2): the window falls back to the reference in
# global memory beyond its LDS margin; the pipeline lag follows the reach R = (19 + 2 SR) / 16 MBs
# (9 at SR 64: 28 diagonals).  Motion of ~100 px per picture puts MVs beyond +-32.
@pytest.mark.parametrize("sr,kw,qp", [
    (48, {}, 28),
    (64, {}, 30),
    (64, dict(restrict_search_range=0), 24),
    (64, dict(transform_8x8_mode=1), 32),
    (64, dict(transform_8x8_mode=1, slice_mbs=7, epzs_dual_refinement=1), 28),
])
def test_epzs_search_range_beyond_32(sr, kw, qp):
    w, h = 320, 240
    pics = moving_seq(w, h, 4, seed=sr + qp, step=(97, -83))
    encode_pair(w, h, pics, [jmhip.JMH_I_SLICE] + [jmhip.JMH_P_SLICE] * 3, qp, search_range=sr, search_mode=3, **kw)


def test_epzs_search_range_64_high10():
    w, h = 320, 240
    pics = hbd_seq(w, h, 4, seed=90, bd=10, step=(-101, 77))
    g = jmhip.Encoder(w, h, search_mode=3, search_range=64, bit_depth=10, transform_8x8_mode=1)
    o = oracle_lib.OracleEncoder(w, h, search_mode=3, search_range=64, bit_depth=10, transform_8x8_mode=1)
    big = 0
    for i, pic in enumerate(pics):
        st = jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE
        gres, grec = g.encode(*pic, st, 30)
        ores, orec = o.encode(*pic, st, 30)
        assert_same(gres, grec, ores, orec, w // 16)
        big += int((np.abs(gres["mv"]) > 4 * 32).sum())
        g.set_reference(*orec)
        o.set_reference(*orec)
    assert big > 0                                      # MVs beyond the SR 32 reach were chosen


@pytest.mark.parametrize("sm", [0, -1])
def test_search_range_beyond_32_needs_epzs(sm):
    with pytest.raises(jmhip.JmhError, match="unsupported configuration"):
        jmhip.Encoder(64, 48, search_range=33, search_mode=sm)


def test_pop_into_equals_pop():
    """The lencod-style pop (results read in place, the deblocked picture into the caller's planes:
    bench.py's host path) returns what pop() + deblocked() return."""
    w, h = 320, 240
    pics = moving_seq(w, h, 6, seed=3, step=(37, -29))
    dbk = (0, 0, 0)
    ref = run_chain(jmhip.Encoder(w, h, search_range=16), pics, 30, dbk, True)
    enc = jmhip.Encoder(w, h, search_range=16)
    planes = (np.empty((h, w), np.uint8), np.empty((h // 2, w // 2), np.uint8), np.empty((h // 2, w // 2), np.uint8))
    got, pending = [], 0
    for i, pic in enumerate(pics):
        if i:
            enc.set_reference_slot(-2)
        if pending == enc.depth:
            got.append((enc.pop_into(*planes).copy(), tuple(p.copy() for p in planes)))
            pending -= 1
        enc.push(*pic, jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE, 30, deblock=dbk)
        pending += 1
    for _ in range(pending):
        got.append((enc.pop_into(*planes).copy(), tuple(p.copy() for p in planes)))
    assert len(got) == len(ref)
    for (gres, gdbk), (rres, _, rdbk) in zip(got, ref):
        assert np.array_equal(gres, rres)
        for x, y in zip(gdbk, rdbk):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("w,h,sr,n,step,kw", [(176, 144, 16, 9, (37, -29), {}), (320, 240, 32, 8, (37, -29), {}),
                                              (1920, 1088, 32, 20, (37, -29), {}), (1920, 1088, 32, 12, (-62, -61), {}),
                                              (640, 480, 32, 10, (63, 62), {}),
                                              (640, 480, 32, 10, (37, -29), dict(search_mode=3, transform_8x8_mode=1)),
                                              (1920, 1088, 32, 20, (-62, -61), dict(search_mode=3, transform_8x8_mode=1)),
                                              # tall: 526 diagonals, ~33 pictures in flight (PMAX entries per tick)
                                              (256, 4096, 32, 40, (37, -29), {}),
                                              (256, 4096, 32, 40, (-62, -61), dict(search_mode=3, transform_8x8_mode=1)),
                                              (1920, 1088, 32, 12, (37, -29), dict(slice_mbs=120)),
                                              (640, 480, 32, 10, (-62, -61), dict(search_mode=3, transform_8x8_mode=1, slice_mbs=57)),
                                              # SearchRange 64 (EPZS): lag 28 diagonals, MVs up to ~128 px
                                              (640, 480, 64, 10, (121, -117), dict(search_mode=3)),
                                              (256, 2048, 64, 24, (-119, 113), dict(search_mode=3, transform_8x8_mode=1))])
def test_pipelined_chain_equals_sequential(w, h, sr, n, step, kw):
    """Pictures in flight together (lag PIPE_LAG diagonals) == one picture at a time, bit for
    bit, under motion that pushes MVs to the search-window edge (|MV| up to 63 px at SR 32: the
    reference is read up to 67 px beyond the MB, the reach PIPE_LAG is derived from)."""
    pics = moving_seq(w, h, n, seed=w + n, step=step)
    dbk = (0, 0, 0)
    a = jmhip.Encoder(w, h, search_range=sr, **kw)                 # auto depth
    b = jmhip.Encoder(w, h, search_range=sr, pipeline_depth=1, **kw)
    assert a.depth > 1 and b.depth == 1
    ra = run_chain(a, pics, 30, dbk, True)
    rb = run_chain(b, pics, 30, dbk, False)
    assert len(ra) == len(rb) == n
    for (gres, grec, gdbk), (ores, orec, odbk) in zip(ra, rb):
        assert_same(gres, grec, ores, orec, w // 16)
        for x, y in zip(gdbk, odbk):
            assert np.array_equal(x, y)
    assert any((r["mb_type"] != 0).any() for r, _, _ in ra[1:])


def test_pipelined_slots_equal_sequential():
    """bench.py's path: encode_slot chain (no readback) pipelined == depth 1 (checked through the
    reference it leaves for a final read-back picture)."""
    w, h = 352, 288
    pics = moving_seq(w, h, 4, seed=5, step=(-21, 13))
    res = []
    for depth in (0, 1):
        e = jmhip.Encoder(w, h, search_range=32, slots=3, pipeline_depth=depth)
        for i in range(3):
            e.load_frame(i, *pics[i])
        e.encode_slot(0, jmhip.JMH_I_SLICE, 28, deblock=(0, 0, 0))
        for k in range(11):
            e.set_reference_slot(-2)
            e.encode_slot(1 + k % 2, jmhip.JMH_P_SLICE, 28, deblock=(0, 0, 0))
        e.set_reference_slot(-2)
        res.append(e.encode(*pics[3], jmhip.JMH_P_SLICE, 28, deblock=(0, 0, 0)) + (e.deblocked(),))
    (gres, grec, gd), (ores, orec, od) = res
    assert_same(gres, grec, ores, orec, w // 16)
    for x, y in zip(gd, od):
        assert np.array_equal(x, y)


# ---------------- High 10 (f5): the EPZS wavefront on 16-bit samples ----------------
def hbd_seq(w, h, n, seed, bd, step=(29, -23)):
    """moving_seq widened to bd bits: samples << (bd - 8) plus low-bit noise, full range used."""
    rng = np.random.default_rng(seed)
    out = []
    for y, u, v in moving_seq(w, h, n, seed, step):
        sh = bd - 8
        out.append(tuple(np.ascontiguousarray((p.astype(np.uint16) << sh) | rng.integers(0, 1 << sh, p.shape, dtype=np.uint16))
                         for p in (y, u, v)))
    return out


@pytest.mark.parametrize("bd,kw,qp,cqp", [
    (10, dict(search_range=16), 28, 0),
    (10, dict(search_range=16, transform_8x8_mode=1), 28, 0),
    (10, dict(search_range=32, transform_8x8_mode=1, restrict_search_range=0), 0, -12),   # QP'c < 12, QPc < 0
    (10, dict(search_range=8), 51, 12),
    (9, dict(search_range=16, transform_8x8_mode=1, use_hadamard=0), 20, 0),
    (10, dict(search_range=16, transform_8x8_mode=1, slice_mbs=5), 30, 0),
    (10, dict(search_range=16, epzs_dual_refinement=1, inter_search=(1, 0, 1, 1, 0, 1, 1)), 36, 3),
])
def test_high10_pictures(bd, kw, qp, cqp):
    """f5: k_mb_epzs / k_mb_intra / k_mb_final on 16-bit samples == the oracle's 16-bit
    restatement on every macroblock (QP'Y, QP'C incl. negative QPc, Clip1 to 2^bd - 1)."""
    w, h = 176, 144
    pics = hbd_seq(w, h, 4, seed=70 + qp, bd=bd)
    g = jmhip.Encoder(w, h, search_mode=3, bit_depth=bd, **kw)
    o = oracle_lib.OracleEncoder(w, h, search_mode=3, bit_depth=bd, **kw)
    for i, pic in enumerate(pics):
        st = jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE
        gres, grec = g.encode(*pic, st, qp, chroma_qp_offset=cqp)
        ores, orec = o.encode(*pic, st, qp, chroma_qp_offset=cqp)
        assert_same(gres, grec, ores, orec, w // 16)
        assert grec[0].dtype == np.uint16 and int(grec[0].max()) < (1 << bd)
        g.set_reference(*orec)
        o.set_reference(*orec)


def test_high10_extremes():
    """Saturated 10-bit content (0 / 1023 checkerboards): Clip1 at both ends, GPU == oracle."""
    rng = np.random.default_rng(8)
    w, h = 64, 48
    pics = [tuple(np.ascontiguousarray((rng.integers(0, 2, s) * 1023).astype(np.uint16)) for s in ((h, w), (h // 2, w // 2), (h // 2, w // 2)))
            for _ in range(3)]
    for qp in (0, 18, 51):
        g = jmhip.Encoder(w, h, search_range=8, search_mode=3, transform_8x8_mode=1, bit_depth=10)
        o = oracle_lib.OracleEncoder(w, h, search_range=8, search_mode=3, transform_8x8_mode=1, bit_depth=10)
        for i, pic in enumerate(pics):
            st = jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE
            gres, grec = g.encode(*pic, st, qp)
            ores, orec = o.encode(*pic, st, qp)
            assert_same(gres, grec, ores, orec, w // 16)
            g.set_reference(*orec)
            o.set_reference(*orec)


def test_high10_config5_width_3840():
    """Config 5's shape at its real width (3840, SliceArgument 240 = one MB row per slice), High 10
    EPZS + 8x8 transform under large motion: GPU == oracle on every macroblock."""
    w, h = 3840, 128
    pics = hbd_seq(w, h, 3, seed=41, bd=10)
    g = jmhip.Encoder(w, h, search_range=32, search_mode=3, transform_8x8_mode=1, slice_mbs=240, bit_depth=10)
    o = oracle_lib.OracleEncoder(w, h, search_range=32, search_mode=3, transform_8x8_mode=1, slice_mbs=240, bit_depth=10)
    for i, pic in enumerate(pics):
        st = jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE
        gres, grec = g.encode(*pic, st, 28)
        ores, orec = o.encode(*pic, st, 28)
        assert_same(gres, grec, ores, orec, w // 16)
        g.set_reference(*orec)
        o.set_reference(*orec)


def test_high10_pipelined_chain_equals_sequential():
    """16-bit pictures in flight together (device deblocking as the reference) == one at a time."""
    w, h, n = 640, 480, 8
    pics = hbd_seq(w, h, n, seed=3, bd=10, step=(-62, -61))
    kw = dict(search_range=32, search_mode=3, transform_8x8_mode=1, bit_depth=10)
    a = jmhip.Encoder(w, h, **kw)
    b = jmhip.Encoder(w, h, pipeline_depth=1, **kw)
    assert a.depth > 1
    ra = run_chain(a, pics, 30, (0, 0, 0), True)
    rb = run_chain(b, pics, 30, (0, 0, 0), False)
    for (gres, grec, gdbk), (ores, orec, odbk) in zip(ra, rb):
        assert_same(gres, grec, ores, orec, w // 16)
        for x, y in zip(gdbk, odbk):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("sm,bd,kw,qp", [
    (0, 10, dict(search_range=16), 28),
    (0, 10, dict(search_range=32, restrict_search_range=0, transform_8x8_mode=1), 20),
    (0, 9, dict(search_range=8, use_hadamard=0, restrict_search_range=1), 40),
    (0, 10, dict(search_range=16, slice_mbs=7, inter_search=(1, 0, 1, 1, 0, 1, 1)), 4),
    (-1, 10, dict(search_range=16), 28),
    (-1, 10, dict(search_range=8, restrict_search_range=0, transform_8x8_mode=1), 51),
    (-1, 9, dict(search_range=16, use_hadamard=0, slice_mbs=11), 12),
])
def test_high10_ffs_and_full_search(sm, bd, kw, qp):
    """16-bit samples through k_mb_me_full<uint16_t, FFS> (SearchMode 0: FastFullPelBlockMotionSearch on the
    MB's common window, SearchMode -1: FullPelBlockMotionSearch) == the oracle on every macroblock
    (VERDICT r3 item 7)."""
    w, h = 176, 144
    pics = hbd_seq(w, h, 4, seed=110 + qp + sm, bd=bd, step=(5, -3))
    g = jmhip.Encoder(w, h, search_mode=sm, bit_depth=bd, **kw)
    o = oracle_lib.OracleEncoder(w, h, search_mode=sm, bit_depth=bd, **kw)
    for i, pic in enumerate(pics):
        st = jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE
        gres, grec = g.encode(*pic, st, qp)
        ores, orec = o.encode(*pic, st, qp)
        assert_same(gres, grec, ores, orec, w // 16)
        g.set_reference(*orec)
        o.set_reference(*orec)


@pytest.mark.parametrize("sm", [0, -1])
def test_high10_ffs_full_width_3840(sm):
    """10-bit FFS / full search at 3840 wide, SR 32, large motion: GPU == oracle."""
    w, h = 3840, 64
    pics = hbd_seq(w, h, 3, seed=47 - sm, bd=10)
    g = jmhip.Encoder(w, h, search_range=32, search_mode=sm, bit_depth=10)
    o = oracle_lib.OracleEncoder(w, h, search_range=32, search_mode=sm, bit_depth=10)
    for i, pic in enumerate(pics):
        st = jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE
        gres, grec = g.encode(*pic, st, 30)
        ores, orec = o.encode(*pic, st, 30)
        assert_same(gres, grec, ores, orec, w // 16)
        g.set_reference(*orec)
        o.set_reference(*orec)


def test_high10_ffs_pipelined_chain_equals_sequential():
    w, h, n = 640, 320, 5
    pics = hbd_seq(w, h, n, seed=4, bd=10, step=(-45, 38))
    kw = dict(search_range=32, search_mode=0, bit_depth=10)
    a = jmhip.Encoder(w, h, **kw)
    b = jmhip.Encoder(w, h, pipeline_depth=1, **kw)
    assert a.depth > 1
    ra = run_chain(a, pics, 30, (0, 0, 0), True)
    rb = run_chain(b, pics, 30, (0, 0, 0), False)
    for (gres, grec, gdbk), (ores, orec, odbk) in zip(ra, rb):
        assert_same(gres, grec, ores, orec, w // 16)
        for x, y in zip(gdbk, odbk):
            assert np.array_equal(x, y)


def test_high10_rejects_other_bit_depths_and_8bit_calls():
    with pytest.raises(jmhip.JmhError):
        jmhip.Encoder(64, 48, search_range=8, search_mode=0, bit_depth=12)
    e = jmhip.Encoder(64, 48, search_range=8, search_mode=3, bit_depth=10)
    y8 = np.zeros((48, 64), np.uint8), np.zeros((24, 32), np.uint8), np.zeros((24, 32), np.uint8)
    assert e.lib.jmh_set_reference(e.ctx, 0, 0, y8[0].ctypes.data, y8[1].ctypes.data, y8[2].ctypes.data, 64, 32) == jmhip.JMH_E_UNSUPPORTED_CFG
    big = [np.full(s, 1024, np.uint16) for s in ((48, 64), (24, 32), (24, 32))]   # out of range for 10 bits
    assert e.lib.jmh_set_reference_u16(e.ctx, 0, 0, big[0].ctypes.data, big[1].ctypes.data, big[2].ctypes.data, 64, 32) == jmhip.JMH_E_INVALID_ARG
    # one sample above 1023 (the last Cr sample) rejects a push / load (checked while packing) and
    # leaves the context usable
    ok = [np.full(s, 1023, np.uint16) for s in ((48, 64), (24, 32), (24, 32))]
    one = [p.copy() for p in ok]
    one[2][23, 31] = 1024
    fp = jmhip.frame_params(jmhip.JMH_I_SLICE, 28, bit_depth=10)
    ptrs = [p.ctypes.data for p in one]
    assert e.lib.jmh_frame_push_u16(e.ctx, *ptrs, 64, 32, ctypes.byref(fp)) == jmhip.JMH_E_INVALID_ARG
    assert e.lib.jmh_load_frame_u16(e.ctx, 0, *ptrs, 64, 32) == jmhip.JMH_E_INVALID_ARG
    res, rec = e.encode(*ok, jmhip.JMH_I_SLICE, 28)
    assert int(rec[0].max()) <= 1023


# ---------------- end to end: lencod bitstream + recon, closed loop ----------------
def run_lencod(binary, out_dir, extra):
    args = [binary, "-p", f"OutputFile={out_dir}/a.264", "-p", f"ReconFile={out_dir}/rec.yuv"]
    for e in extra:
        args += ["-p", e]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("extra", [
    ["InputFile=synthetic:1", "FramesToBeEncoded=10", "SourceWidth=176", "SourceHeight=144", "SearchRange=16"],
    ["InputFile=synthetic:2", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "IntraPeriod=3", "QPRemainingFrame=33"],
    ["InputFile=synthetic:3", "FramesToBeEncoded=3", "SourceWidth=200", "SourceHeight=120", "SearchRange=8",
     "LoopFilterParametersFlag=1", "LoopFilterAlphaC0Offset=2", "LoopFilterBetaOffset=-1"],
    ["InputFile=synthetic:4", "FramesToBeEncoded=3", "SourceWidth=176", "SourceHeight=144", "SearchRange=8",
     "LoopFilterParametersFlag=1", "LoopFilterDisable=1"],
    ["InputFile=synthetic:6", "FramesToBeEncoded=5", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "PipelineDepth=1"],
    # config 1: SearchMode -1 (FullPelBlockMotionSearch), QCIF, SR 16
    ["InputFile=synthetic:7", "FramesToBeEncoded=4", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "SearchMode=-1"],
    ["InputFile=synthetic:8", "FramesToBeEncoded=3", "SourceWidth=320", "SourceHeight=240", "SearchRange=8",
     "SearchMode=-1", "RestrictSearchRange=0", "UseHadamard=0"],
    ["InputFile=synthetic:5", "FramesToBeEncoded=4", "SourceWidth=320", "SourceHeight=240", "SearchRange=16",
     "LoopFilterParametersFlag=1", "LoopFilterAlphaC0Offset=6", "LoopFilterBetaOffset=6", "QPFirstFrame=40",
     "QPRemainingFrame=44"],
    # config 3 shape at CIF: High profile, 8x8 transform (a12) + EPZS (a15), pipelined
    ["InputFile=synthetic:23", "FramesToBeEncoded=8", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3"],
    ["InputFile=synthetic:24", "FramesToBeEncoded=5", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "SearchMode=3", "RestrictSearchRange=0", "QPRemainingFrame=34"],
    # High profile, 8x8 transform (a12): pipelined, device deblocking without 4x4 luma edges
    ["InputFile=synthetic:21", "FramesToBeEncoded=8", "SourceWidth=352", "SourceHeight=288", "SearchRange=16",
     "ProfileIDC=100", "Transform8x8Mode=1"],
    ["InputFile=synthetic:22", "FramesToBeEncoded=4", "SourceWidth=200", "SourceHeight=120", "SearchRange=8",
     "ProfileIDC=100", "Transform8x8Mode=1", "QPFirstFrame=38", "QPRemainingFrame=40", "IntraPeriod=2",
     "LoopFilterParametersFlag=1", "LoopFilterAlphaC0Offset=-3", "LoopFilterBetaOffset=2"],
    # JMVersion 10 (docs/JM_SEMANTICS.md item 45): q_offsets.c flat offsets 682 / 342, Intra16x16 in P
    ["InputFile=synthetic:25", "FramesToBeEncoded=4", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "JMVersion=10", "QPRemainingFrame=30"],
    ["InputFile=synthetic:26", "FramesToBeEncoded=5", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3", "JMVersion=10"],
    ["InputFile=synthetic:27", "FramesToBeEncoded=5", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3", "JMVersion=10", "EPZSDualRefinement=1"],
    # SliceMode 1: one NAL unit per slice, neighbours limited to the slice (pipelined, writer threads)
    ["InputFile=synthetic:28", "FramesToBeEncoded=5", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "SliceMode=1", "SliceArgument=22"],
    ["InputFile=synthetic:29", "FramesToBeEncoded=4", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "SliceMode=1", "SliceArgument=7", "IntraPeriod=2", "WriterThreads=0"],
    ["InputFile=synthetic:30", "FramesToBeEncoded=5", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3", "SliceMode=1", "SliceArgument=40"],
    ["InputFile=synthetic:31", "FramesToBeEncoded=3", "SourceWidth=176", "SourceHeight=144", "SearchRange=8",
     "SearchMode=-1", "SliceMode=1", "SliceArgument=1"],
    # CABAC (SymbolMode 1, row f4): pipelined device backend + writer threads, Main and High
    ["InputFile=synthetic:32", "FramesToBeEncoded=8", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=77", "SymbolMode=1", "IntraPeriod=4"],
    ["InputFile=synthetic:33", "FramesToBeEncoded=6", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3", "SymbolMode=1", "SliceMode=1", "SliceArgument=22"],
    ["InputFile=synthetic:34", "FramesToBeEncoded=4", "SourceWidth=176", "SourceHeight=144", "SearchRange=8",
     "ProfileIDC=77", "SymbolMode=1", "SearchMode=-1", "QPFirstFrame=0", "QPRemainingFrame=2", "WriterThreads=0"],
    # High 10 (f5, ProfileIDC 110): the pipelined 16-bit wavefront, CAVLC and CABAC, slices
    ["InputFile=synthetic:35", "FramesToBeEncoded=8", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SearchMode=3"],
    ["InputFile=synthetic:36", "FramesToBeEncoded=6", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SearchMode=3",
     "SymbolMode=1", "SliceMode=1", "SliceArgument=22", "IntraPeriod=3"],
    ["InputFile=synthetic:37", "FramesToBeEncoded=4", "SourceWidth=200", "SourceHeight=120", "SearchRange=16",
     "ProfileIDC=110", "SourceBitDepthLuma=9", "SourceBitDepthChroma=9", "SearchMode=3", "QPFirstFrame=2",
     "QPRemainingFrame=4", "ChromaQPOffset=-10", "WriterThreads=0"],
    # High 10 with FFS / full search
    ["InputFile=synthetic:38", "FramesToBeEncoded=5", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SearchMode=0"],
    ["InputFile=synthetic:39", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=16",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "SearchMode=-1", "SymbolMode=1",
     "SliceMode=1", "SliceArgument=22"],
    # SearchRange 64 with EPZS (the pipelined lencod, lag 28)
    ["InputFile=synthetic:40", "FramesToBeEncoded=6", "SourceWidth=352", "SourceHeight=288", "SearchRange=64",
     "SearchMode=3", "ProfileIDC=100", "Transform8x8Mode=1"],
])
def test_lencod_bitstream_identical(extra):
    with tempfile.TemporaryDirectory() as a, tempfile.TemporaryDirectory() as b:
        run_lencod(LENCOD, a, extra)
        run_lencod(LENCOD_CPU, b, extra)
        ga, oa = open(f"{a}/a.264", "rb").read(), open(f"{b}/a.264", "rb").read()
        assert ga == oa, "bitstreams differ"
        assert open(f"{a}/rec.yuv", "rb").read() == open(f"{b}/rec.yuv", "rb").read()
        r = subprocess.run([JMDEC, f"{a}/a.264", f"{a}/dec.yuv"], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        assert open(f"{a}/dec.yuv", "rb").read() == open(f"{a}/rec.yuv", "rb").read()


# UseConstrainedIntraPred 1 (constrained_intra_pred_flag): the device's intra availability
# (intra_avail: inter neighbours not available for intra prediction, their 4x4 modes not for the mode
# prediction) == the oracle's, through the whole lencod (tick FFS path, full search, EPZS + High +
# slices, CABAC, RDO 8 / 10 bit); each case also differs from its UseConstrainedIntraPred 0 encoding
@pytest.mark.parametrize("extra", [
    ["InputFile=synthetic:81", "FramesToBeEncoded=5", "SourceWidth=176", "SourceHeight=144", "SearchRange=2",
     "QPRemainingFrame=20"],
    ["InputFile=synthetic:82", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=8",
     "ProfileIDC=77", "SymbolMode=1", "QPRemainingFrame=40"],
    ["InputFile=synthetic:83", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=4",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3", "SliceMode=1", "SliceArgument=22", "QPRemainingFrame=24"],
    ["InputFile=synthetic:86", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=8",
     "ProfileIDC=100", "Transform8x8Mode=1", "QPRemainingFrame=26"],
    ["InputFile=synthetic:87", "FramesToBeEncoded=4", "SourceWidth=176", "SourceHeight=144", "SearchRange=4",
     "SearchMode=-1", "QPRemainingFrame=30"],
    ["InputFile=synthetic:84", "FramesToBeEncoded=3", "SourceWidth=352", "SourceHeight=288", "SearchRange=8",
     "RDOptimization=1", "SymbolMode=1", "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3", "QPRemainingFrame=30"],
    ["InputFile=synthetic:85", "FramesToBeEncoded=3", "SourceWidth=352", "SourceHeight=288", "SearchRange=8",
     "RDOptimization=1", "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "SearchMode=3",
     "QPRemainingFrame=44"],
], ids=["ffs", "cabac", "high_epzs_slices", "high_ffs", "full", "rdo_t8", "rdo_high10"])
def test_lencod_constrained_intra(extra):
    test_lencod_bitstream_identical(extra + ["UseConstrainedIntraPred=1"])
    with tempfile.TemporaryDirectory() as a, tempfile.TemporaryDirectory() as b:
        run_lencod(LENCOD_CPU, a, extra + ["UseConstrainedIntraPred=1"])
        run_lencod(LENCOD_CPU, b, extra)
        assert open(f"{a}/rec.yuv", "rb").read() != open(f"{b}/rec.yuv", "rb").read()


@pytest.mark.slow
def test_1080p_closed_loop_gpu():
    """Full config-2 size: GPU bitstream decodes to exactly the GPU reconstruction."""
    extra = ["InputFile=synthetic:0", "FramesToBeEncoded=6", "SourceWidth=1920", "SourceHeight=1080", "SearchRange=32"]
    with tempfile.TemporaryDirectory() as a:
        run_lencod(LENCOD, a, extra)
        r = subprocess.run([JMDEC, f"{a}/a.264", f"{a}/dec.yuv"], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr
        assert open(f"{a}/dec.yuv", "rb").read() == open(f"{a}/rec.yuv", "rb").read()


@pytest.mark.slow
def test_1080p_p_frame_parity():
    """One full 1080p (coded 1920x1088) P picture, FFS SR=32: GPU == oracle on every MB."""
    w, h = 1920, 1088
    pics = [jmhip.synth_frame(1920, 1080, 0, i) for i in range(2)]
    g = jmhip.Encoder(w, h, search_range=32)
    o = oracle_lib.OracleEncoder(w, h, search_range=32)
    g.set_reference(*pics[0])
    o.set_reference(*pics[0])
    gres, grec = g.encode(*pics[1], jmhip.JMH_P_SLICE, 28)
    ores, orec = o.encode(*pics[1], jmhip.JMH_P_SLICE, 28)
    assert_same(gres, grec, ores, orec, w // 16)


@pytest.mark.slow
def test_config3_2160p_parity():
    """BASELINE config 3 at its full size: 3840x2160 High profile, EPZS SR 32 +
    Transform8x8Mode 1, the bench's synthetic stream 0 (IDR + P): GPU == oracle on every macroblock
    and every reconstructed sample (the oracle takes ~10 s per picture)."""
    w, h = 3840, 2160
    pics = [jmhip.synth_frame(w, h, 0, i) for i in range(2)]
    encode_pair(w, h, pics, [jmhip.JMH_I_SLICE, jmhip.JMH_P_SLICE], 28, search_range=32, search_mode=3,
                transform_8x8_mode=1)

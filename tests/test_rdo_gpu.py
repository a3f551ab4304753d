"""RDOptimization = 1 on the MI355X (row f4, config 5): k_rdo_inter / k_rdo_intra / k_rdo_final on the RD stage
schedule must equal the CPU oracle (oracle/rdo.c) bit for bit -- every macroblock's result
(mode, MVs, levels, the chosen candidate's rate in min_cost) and the reconstruction -- and the
product lencod with the device RD loop must write the same bitstream as the CPU lencod, with the
writer's RD rate check at 0 mismatches.  JM parity of the RD choices is unpinned
(docs/JM_SEMANTICS.md items 53-60, 63; SymbolMode 0, the CAVLC rates: item 64)."""
import tempfile

import numpy as np
import pytest

import oracle_lib
from jmpaths import LENCOD, LENCOD_CPU, ensure_built, load_jmhip
from test_gpu_parity import assert_same, hbd_seq, moving_seq, run_chain, run_lencod, synth_seq

jmhip = load_jmhip()
pytestmark = pytest.mark.gpu

RDO = dict(rdo=1, symbol_mode=1, search_mode=3)


@pytest.fixture(scope="module", autouse=True)
def built():
    ensure_built()
    jmhip.load()


def rdo_pair(w, h, pics, qp, cqp=0, bd=8, symbol_mode=1, stats=None, **kw):
    """GPU == oracle on every picture; returns the last picture's results, and with stats (a dict)
    counts the 8x8-transform macroblocks of all pictures into stats["t8"]"""
    kw = dict(RDO, **kw, symbol_mode=symbol_mode)
    g = jmhip.Encoder(w, h, bit_depth=bd, **kw)
    o = oracle_lib.OracleEncoder(w, h, bit_depth=bd, **kw)
    for i, pic in enumerate(pics):
        st = jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE
        gres, grec = g.encode(*pic, st, qp, chroma_qp_offset=cqp)
        ores, orec = o.encode(*pic, st, qp, chroma_qp_offset=cqp)
        assert_same(gres, grec, ores, orec, w // 16)
        # every MB reports its rate in bits (a P_Skip can cost 0 bits: an MPS bin with no renormalisation)
        assert (gres["min_cost"] >= 0).all() and gres["min_cost"].sum() > 0
        g.set_reference(*orec)
        o.set_reference(*orec)
        if stats is not None:
            stats["t8"] = stats.get("t8", 0) + int((gres["transform_8x8"] != 0).sum())
    return gres


def test_rdo_qcif_ipp():
    pics = synth_seq(176, 144, 4, 71)
    res = rdo_pair(176, 144, pics, 28, search_range=16)
    assert len(set(res["mb_type"].tolist())) > 2      # several modes actually compete


@pytest.mark.parametrize("kw,qp,cqp", [
    (dict(search_range=8), 0, 0),
    (dict(search_range=8), 51, 0),
    (dict(search_range=16, slice_mbs=11), 36, -5),
    (dict(search_range=8, slice_mbs=1), 28, 0),
    (dict(search_range=8, use_hadamard=0, restrict_search_range=0), 24, 0),
    (dict(search_range=8, inter_search=(0, 1, 1, 1, 0, 1, 1), epzs_dual_refinement=1), 20, 3),
    (dict(search_range=4, inter_search=(1, 0, 0, 0, 0, 0, 0)), 30, 0),
    (dict(search_range=16, jm_version=10), 31, 0),
])
def test_rdo_configs(kw, qp, cqp):
    pics = moving_seq(176, 144, 3, seed=80 + qp)
    rdo_pair(176, 144, pics, qp, cqp, **kw)


@pytest.mark.parametrize("bd,qp,cqp", [(10, 28, 0), (9, 4, -12), (10, 51, 12)])
def test_rdo_high10(bd, qp, cqp):
    pics = hbd_seq(176, 144, 3, seed=90 + qp, bd=bd)
    rdo_pair(176, 144, pics, qp, cqp, bd=bd, search_range=16, slice_mbs=11)


def test_rdo_config5_width_3840():
    """Config 5's shape at its real width: High 10, one MB row per slice (SliceArgument 240), EPZS
    SR 32, RDO on: the stage schedule is the diagonal wavefront, 240-MB CABAC chains per slice."""
    w, h = 3840, 96
    pics = hbd_seq(w, h, 3, seed=43, bd=10)
    rdo_pair(w, h, pics, 28, bd=10, search_range=32, slice_mbs=240)


# ---- Transform8x8Mode 1 with RDO on (docs/JM_SEMANTICS.md item 63): I8MB by RDCost_for_8x8IntraBlocks,
#      16x16 / 16x8 / 8x16 / all-8x8 P8x8 each also with transform_size_8x8_flag 1
@pytest.mark.parametrize("kw,qp,cqp", [
    (dict(search_range=16), 28, 0),
    (dict(search_range=8), 8, 0),                          # no 8x8 transform wins here (oracle alike)
    (dict(search_range=8), 44, -3),
    (dict(search_range=16, slice_mbs=11), 34, 2),
    (dict(search_range=8, inter_search=(1, 1, 1, 1, 0, 0, 0), jm_version=10), 24, 0),   # P8x8 = all 8x8
])
def test_rdo_t8_configs(kw, qp, cqp):
    pics = moving_seq(176, 144, 3, seed=60 + qp)
    st = {}
    rdo_pair(176, 144, pics, qp, cqp, transform_8x8_mode=1, stats=st, **kw)
    assert st["t8"] > 0 or qp < 10


@pytest.mark.parametrize("bd,qp", [(10, 28), (9, 6)])
def test_rdo_t8_high10(bd, qp):
    pics = hbd_seq(176, 144, 3, seed=95 + qp, bd=bd)
    rdo_pair(176, 144, pics, qp, 0, bd=bd, search_range=16, slice_mbs=11, transform_8x8_mode=1)


def test_rdo_t8_config5_width_3840():
    """Config 5 with Transform8x8Mode 1 at its real width: High 10, one MB row per slice, EPZS SR 32,
    RDO on with the 8x8-transform candidates and I8MB."""
    w, h = 3840, 96
    pics = hbd_seq(w, h, 3, seed=44, bd=10)
    st = {}
    rdo_pair(w, h, pics, 28, bd=10, search_range=32, slice_mbs=240, transform_8x8_mode=1, stats=st)
    assert st["t8"] > 0


# ---- SymbolMode 0 (docs/JM_SEMANTICS.md item 64): the RD rate is the CAVLC bit count (nC from the
#      neighbours' and the decided blocks' TotalCoeff, the slice's mb_skip_run before a coded MB)
@pytest.mark.parametrize("kw,qp,cqp", [
    (dict(search_range=16), 28, 0),
    (dict(search_range=8), 0, 0),                                   # long level codes (escapes)
    (dict(search_range=8, slice_mbs=1), 48, 0),                     # runs reset at every slice
    (dict(search_range=16, slice_mbs=11), 34, 4),
    (dict(search_range=8, inter_search=(0, 1, 1, 1, 0, 1, 1), use_hadamard=0), 24, 0),
    (dict(search_range=16, transform_8x8_mode=1), 30, 0),
    (dict(search_range=8, transform_8x8_mode=1, jm_version=10), 4, -2),
])
def test_rdo_cavlc_configs(kw, qp, cqp):
    pics = moving_seq(176, 144, 3, seed=30 + qp)
    rdo_pair(176, 144, pics, qp, cqp, symbol_mode=0, **kw)


@pytest.mark.parametrize("bd,t8", [(10, 0), (10, 1), (9, 0)])
def test_rdo_cavlc_high10(bd, t8):
    pics = hbd_seq(176, 144, 3, seed=33 + bd, bd=bd)
    rdo_pair(176, 144, pics, 26, 0, bd=bd, symbol_mode=0, search_range=16, slice_mbs=11, transform_8x8_mode=t8)


def test_rdo_cavlc_config5_width_3840():
    """Config 5's shape with SymbolMode 0: High 10, one MB row per slice, EPZS SR 32, CAVLC rates."""
    w, h = 3840, 96
    pics = hbd_seq(w, h, 3, seed=45, bd=10)
    rdo_pair(w, h, pics, 28, bd=10, symbol_mode=0, search_range=32, slice_mbs=240)


# ---- SearchMode 0 (FFS) / -1 (full search) under RDO (item 65): FFS from the MB's shared SAD table
#      (SetupFastFullPelSearch), full search scanning every position of the window on a lane stride;
#      no (0,0) pre-check, no zero-vector bias
@pytest.mark.parametrize("sm,bd,kw,qp", [
    (0, 8, dict(search_range=16), 28),
    (0, 8, dict(search_range=8, slice_mbs=11, transform_8x8_mode=1), 36),
    (-1, 8, dict(search_range=8, restrict_search_range=0), 20),
    (0, 10, dict(search_range=16, symbol_mode=0), 30),
    (-1, 10, dict(search_range=8, transform_8x8_mode=1), 26),
    # SR 32: the SAD table's full 65 x 65 grid (a column past the 64 lanes), MB centres near the edges
    (0, 8, dict(search_range=32), 28),
    (0, 10, dict(search_range=32, restrict_search_range=0, slice_mbs=33), 32),
])
def test_rdo_ffs_full_search(sm, bd, kw, qp):
    pics = (hbd_seq(176, 144, 3, seed=120 + qp, bd=bd) if bd > 8 else moving_seq(176, 144, 3, seed=120 + qp))
    kw = dict(kw)
    symbol_mode = kw.pop("symbol_mode", 1)
    rdo_pair(176, 144, pics, qp, 0, bd=bd, symbol_mode=symbol_mode, search_mode=sm, **kw)


def test_rdo_ffs_width_3840():
    """RDO + FFS at 3840 wide with one-row slices, SR 32 (many positions outside k_rdo_inter's window)."""
    w, h = 3840, 64
    pics = hbd_seq(w, h, 3, seed=48, bd=10)
    rdo_pair(w, h, pics, 28, bd=10, search_range=32, slice_mbs=240, search_mode=0)


@pytest.mark.parametrize("slice_mbs", [40, 0, 100])
def test_rdo_pipelined_chain_equals_sequential(slice_mbs):
    """Pictures in flight on the RD stage schedule (one-row slices: diagonals, lag 16; one slice
    per picture: raster order, lag 5 mbw + 6; 100-MB slices straddling rows) with the device-
    deblocked reference == one picture at a time."""
    w, h, n = 640, 320, 5
    pics = moving_seq(w, h, n, seed=5, step=(-45, 38))
    kw = dict(search_range=32, slice_mbs=slice_mbs, **RDO)
    a = jmhip.Encoder(w, h, **kw)
    b = jmhip.Encoder(w, h, pipeline_depth=1, **kw)
    assert a.depth > 1
    ra = run_chain(a, pics, 30, (0, 0, 0), True)
    rb = run_chain(b, pics, 30, (0, 0, 0), False)
    for (gres, grec, gdbk), (ores, orec, odbk) in zip(ra, rb):
        assert_same(gres, grec, ores, orec, w // 16)
        for x, y in zip(gdbk, odbk):
            assert np.array_equal(x, y)


def test_rdo_search_range_64():
    """RDOptimization 1 with EPZS at SearchRange 64: GPU == oracle, and the RD stage schedule's
    lag from the reach (9 MBs) keeps pictures in flight == one at a time."""
    w, h = 320, 240
    pics = moving_seq(w, h, 4, seed=64, step=(97, -83))
    rdo_pair(w, h, pics, 30, search_range=64, search_mode=3, slice_mbs=20)
    kw = dict(search_range=64, slice_mbs=20, **RDO)
    a = jmhip.Encoder(w, h, **kw)
    b = jmhip.Encoder(w, h, pipeline_depth=1, **kw)
    assert a.depth > 1
    ra = run_chain(a, pics, 30, (0, 0, 0), True)
    rb = run_chain(b, pics, 30, (0, 0, 0), False)
    for (gres, grec, gdbk), (ores, orec, odbk) in zip(ra, rb):
        assert_same(gres, grec, ores, orec, w // 16)
        for x, y in zip(gdbk, odbk):
            assert np.array_equal(x, y)


def test_rdo_slot_chain_varying_qp():
    """an encode_slot chain with RDO on, a different QP (so different lambdas) per
    picture and more pictures than the context's ring (depth + 2 entries): every picture's lambdas
    are staged through its ring entry's pinned buffer while earlier pictures are still in flight.
    Pipelined == one picture at a time, checked through the reference the chain leaves for a
    final read-back picture, for CABAC and CAVLC rates."""
    w, h = 352, 96
    pics = moving_seq(w, h, 4, seed=7, step=(-9, 5))
    qps = [22, 34, 27, 40, 25]
    for symbol_mode in (1, 0):
        res = []
        for depth in (0, 1):
            e = jmhip.Encoder(w, h, search_range=16, slots=3, pipeline_depth=depth, slice_mbs=22,
                              **dict(RDO, symbol_mode=symbol_mode))
            if depth == 0:
                assert e.depth > 1
            for i in range(3):
                e.load_frame(i, *pics[i])
            e.encode_slot(0, jmhip.JMH_I_SLICE, 26, deblock=(0, 0, 0))
            for k in range(13):
                e.set_reference_slot(-2)
                e.encode_slot(1 + k % 2, jmhip.JMH_P_SLICE, qps[k % len(qps)], deblock=(0, 0, 0))
            e.set_reference_slot(-2)
            res.append(e.encode(*pics[3], jmhip.JMH_P_SLICE, 30, deblock=(0, 0, 0)) + (e.deblocked(),))
        (gres, grec, gd), (ores, orec, od) = res
        assert_same(gres, grec, ores, orec, w // 16)
        for x, y in zip(gd, od):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("extra", [
    ["InputFile=synthetic:71", "FramesToBeEncoded=5", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "ProfileIDC=77"],
    ["InputFile=synthetic:72", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=77", "SliceMode=1", "SliceArgument=22", "IntraPeriod=3", "QPRemainingFrame=33"],
    ["InputFile=synthetic:73", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=16",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "SliceMode=1", "SliceArgument=22",
     "LoopFilterParametersFlag=1", "LoopFilterAlphaC0Offset=2", "LoopFilterBetaOffset=-1"],
    ["InputFile=synthetic:74", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=16",
     "ProfileIDC=100", "Transform8x8Mode=1", "IntraPeriod=3"],
    ["InputFile=synthetic:75", "FramesToBeEncoded=3", "SourceWidth=352", "SourceHeight=96", "SearchRange=32",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SliceMode=1",
     "SliceArgument=22"],
    # SearchMode 0 / -1 under RDO (item 65)
    ["InputFile=synthetic:78", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=16",
     "ProfileIDC=77", "SearchMode=0"],
    ["InputFile=synthetic:79", "FramesToBeEncoded=3", "SourceWidth=176", "SourceHeight=144", "SearchRange=8",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=-1", "SymbolMode=0"],
    # SymbolMode 0 (item 64)
    ["InputFile=synthetic:76", "FramesToBeEncoded=5", "SourceWidth=352", "SourceHeight=288", "SearchRange=16",
     "ProfileIDC=66", "SymbolMode=0"],
    ["InputFile=synthetic:77", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=96", "SearchRange=32",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SliceMode=1",
     "SliceArgument=22", "SymbolMode=0", "QPRemainingFrame=40"],
])
def test_rdo_lencod_bitstream_identical(extra):
    """The product lencod (device RD loop, device deblocking, pipelined pictures, writer threads)
    and the CPU lencod write identical bitstreams and reconstructions; both writers check every
    macroblock's RD rate against the CABAC / CAVLC bits they emit."""
    args = ["SymbolMode=1", "SearchMode=3"] + extra + ["RDOptimization=1"]   # later entries win
    with tempfile.TemporaryDirectory() as g, tempfile.TemporaryDirectory() as c:
        lg = run_lencod(LENCOD, g, args)
        lc = run_lencod(LENCOD_CPU, c, args)
        for log in (lg, lc):
            assert "RD rate check:" in log and ", 0 whose RD rate differs" in log, log
        assert open(f"{g}/a.264", "rb").read() == open(f"{c}/a.264", "rb").read()
        assert open(f"{g}/rec.yuv", "rb").read() == open(f"{c}/rec.yuv", "rb").read()


def test_rdo_rejects_unsupported():
    for kw in (dict(rdo=1, symbol_mode=2, search_mode=3), dict(rdo=2, symbol_mode=1, search_mode=3),
               dict(rdo=1, symbol_mode=0, search_mode=2)):
        with pytest.raises(jmhip.JmhError):
            jmhip.Encoder(64, 48, search_range=8, **kw)


@pytest.mark.parametrize("slice_mbs,bd", [(0, 8), (11, 8), (0, 10)])
def test_rdo_cavlc_last_mb_skip(slice_mbs, bd):
    """docs/JM_SEMANTICS.md item 64(a) on the device: flat pictures (every P macroblock skipped); the
    last macroblock's skip carries ue(mb_skip_run + 1), every other skip 0 bits -- GPU == oracle"""
    w, h = 176, 144
    nmb = (w // 16) * (h // 16)
    dt = np.uint16 if bd > 8 else np.uint8
    mid = 1 << (bd - 1)
    pic = (np.full((h, w), mid, dt), np.full((h // 2, w // 2), mid, dt), np.full((h // 2, w // 2), mid, dt))
    res = rdo_pair(w, h, [pic] * 3, 28, bd=bd, symbol_mode=0, search_range=8, slice_mbs=slice_mbs)
    mt, mc = res["mb_type"].tolist(), res["min_cost"].tolist()
    assert mt.count(0) == nmb
    run = (nmb - 1) % (slice_mbs or nmb)
    assert mc[-1] == 2 * (run + 2).bit_length() - 1 and not any(mc[:-1])


@pytest.mark.slow
def test_rdo_config5_2160p_parity():
    """BASELINE config 5 at its full size: 3840x2160 High 10, EPZS SR 32, CABAC
    RDOptimization 1, 240-MB (one-row) slices, the bench's synthetic 10-bit stream 0 (IDR + P):
    GPU == oracle on every macroblock, rate and reconstructed sample."""
    w, h = 3840, 2160
    pics = [jmhip.synth_frame(w, h, 0, i, bit_depth=10) for i in range(2)]
    rdo_pair(w, h, pics, 28, bd=10, search_range=32, slice_mbs=240)

"""RDOptimization = 1: encode_one_macroblock's rate-distortion loop
(RDCost_for_macroblocks / RDCost_for_8x8blocks / RDCost_for_4x4IntraBlocks [J]) with the CABAC rate
of csrc/jmh_cabac_rate.h, on the CPU oracle (oracle/rdo.c) through the product's host plumbing.

Pinned here (CPU):
  * the closed loop: the independent decoder reproduces the RD encoder's reconstruction;
  * the rate: every committed macroblock's RD rate (jmh_mb_result.min_cost) equals the bits the
    product's CABAC writer (host/cabac.c, an independent implementation checked by the decoder)
    emits for it -- lencod prints "RD rate check" and fails on a mismatch;
  * the configuration gate (PatchInp).
JM parity of the RD choices is unpinned (no JM source here; docs/JM_SEMANTICS.md items 53-60)."""
import re
import subprocess
import tempfile

import pytest

from jmpaths import JMDEC, LENCOD_CPU, ensure_built

BASE = ["SymbolMode=1", "RDOptimization=1", "SearchMode=3"]
RDO = [
    ["InputFile=synthetic:71", "FramesToBeEncoded=4", "ProfileIDC=77", "SearchRange=16"],
    ["InputFile=synthetic:72", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=8", "IntraPeriod=1"],
    ["InputFile=synthetic:73", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=4", "QPFirstFrame=0",
     "QPRemainingFrame=0"],
    ["InputFile=synthetic:74", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=4", "QPFirstFrame=51",
     "QPRemainingFrame=51"],
    ["InputFile=synthetic:75", "FramesToBeEncoded=4", "ProfileIDC=77", "SearchRange=16", "SliceMode=1",
     "SliceArgument=11", "ChromaQPOffset=-5", "QPRemainingFrame=36"],
    ["InputFile=synthetic:76", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=8", "SliceMode=1",
     "SliceArgument=1", "SourceWidth=200", "SourceHeight=120", "UseHadamard=0"],
    ["InputFile=synthetic:77", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=8", "InterSearch16x16=0",
     "InterSearch8x4=0", "RestrictSearchRange=0", "EPZSDualRefinement=1", "QPFirstFrame=12", "QPRemainingFrame=20"],
    ["InputFile=synthetic:78", "FramesToBeEncoded=4", "ProfileIDC=77", "SearchRange=16", "SourceWidth=352",
     "SourceHeight=288", "QPRemainingFrame=31", "JMVersion=10"],
    # config 5's sample path: High 10, one MB row per slice
    ["InputFile=synthetic:79", "FramesToBeEncoded=4", "ProfileIDC=110", "SourceBitDepthLuma=10",
     "SourceBitDepthChroma=10", "SearchRange=16", "SliceMode=1", "SliceArgument=11", "IntraPeriod=3"],
    ["InputFile=synthetic:80", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=9",
     "SourceBitDepthChroma=9", "SearchRange=8", "QPFirstFrame=2", "QPRemainingFrame=4", "ChromaQPOffset=-12"],
    # Transform8x8Mode 1 (item 63): I8MB by RDCost_for_8x8IntraBlocks, each inter candidate with the 8x8 transform
    ["InputFile=synthetic:89", "FramesToBeEncoded=4", "ProfileIDC=100", "Transform8x8Mode=1", "SearchRange=16"],
    ["InputFile=synthetic:90", "FramesToBeEncoded=3", "ProfileIDC=100", "Transform8x8Mode=1", "SearchRange=8",
     "IntraPeriod=1", "QPFirstFrame=20"],
    ["InputFile=synthetic:91", "FramesToBeEncoded=4", "ProfileIDC=110", "SourceBitDepthLuma=10",
     "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SearchRange=16", "SliceMode=1", "SliceArgument=11",
     "QPRemainingFrame=24", "JMVersion=10"],
    # SearchMode 0 (FFS) and -1 (full search) under RDO (item 65): no (0,0) pre-check, no zero bias
    ["InputFile=synthetic:99", "FramesToBeEncoded=4", "ProfileIDC=77", "SearchRange=16", "SearchMode=0"],
    ["InputFile=synthetic:100", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=8", "SearchMode=-1",
     "SliceMode=1", "SliceArgument=11", "RestrictSearchRange=0"],
    ["InputFile=synthetic:101", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=10",
     "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SearchRange=16", "SearchMode=0", "UseHadamard=0"],
    ["InputFile=synthetic:102", "FramesToBeEncoded=3", "ProfileIDC=100", "Transform8x8Mode=1", "SearchRange=8",
     "SearchMode=-1", "QPFirstFrame=40", "QPRemainingFrame=44"],
]


def encode(d, extra, name="a"):
    args = [LENCOD_CPU, "-p", f"OutputFile={d}/{name}.264", "-p", f"ReconFile={d}/{name}.yuv"]
    for e in extra:
        args += ["-p", e]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def rate_check(log):
    m = re.search(r"RD rate check: (\d+) macroblocks, (\d+) whose", log)
    assert m, log
    return int(m.group(1)), int(m.group(2))


@pytest.mark.parametrize("extra", RDO, ids=[c[0].split(":")[1] for c in RDO])
def test_rdo_closed_loop_and_rate(extra):
    ensure_built()
    with tempfile.TemporaryDirectory() as d:
        log = encode(d, BASE + extra)
        n, bad = rate_check(log)
        assert n > 0 and bad == 0, log
        r = subprocess.run([JMDEC, f"{d}/a.264", f"{d}/dec.yuv"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(f"{d}/dec.yuv", "rb").read() == open(f"{d}/a.yuv", "rb").read()


# SymbolMode 0 (docs/JM_SEMANTICS.md item 64): the RD loop with CAVLC rates -- JM's default encoder.cfg
# shape (RDOptimization 1, CAVLC), Baseline / Main / High / High 10
CAVLC = [
    ["InputFile=synthetic:92", "FramesToBeEncoded=4", "ProfileIDC=66", "SearchRange=16"],
    ["InputFile=synthetic:93", "FramesToBeEncoded=3", "ProfileIDC=66", "SearchRange=8", "QPFirstFrame=0", "QPRemainingFrame=2"],
    ["InputFile=synthetic:94", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=8", "QPFirstFrame=51",
     "QPRemainingFrame=48", "SliceMode=1", "SliceArgument=1"],
    ["InputFile=synthetic:95", "FramesToBeEncoded=4", "ProfileIDC=100", "Transform8x8Mode=1", "SearchRange=16",
     "SliceMode=1", "SliceArgument=11", "ChromaQPOffset=4"],
    ["InputFile=synthetic:96", "FramesToBeEncoded=3", "ProfileIDC=100", "Transform8x8Mode=1", "SearchRange=8",
     "QPFirstFrame=0", "QPRemainingFrame=0", "IntraPeriod=2"],          # large 8x8 levels: level_prefix > 15
    ["InputFile=synthetic:97", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=10",
     "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SearchRange=16", "QPRemainingFrame=20", "JMVersion=10"],
    ["InputFile=synthetic:98", "FramesToBeEncoded=3", "ProfileIDC=66", "SearchRange=8", "SourceWidth=200",
     "SourceHeight=120", "InterSearch8x4=0", "InterSearch4x8=0", "UseHadamard=0"],
]


@pytest.mark.parametrize("extra", CAVLC, ids=[c[0].split(":")[1] for c in CAVLC])
def test_rdo_cavlc_closed_loop_and_rate(extra):
    ensure_built()
    with tempfile.TemporaryDirectory() as d:
        log = encode(d, ["SymbolMode=0", "RDOptimization=1", "SearchMode=3"] + extra)
        n, bad = rate_check(log)
        assert n > 0 and bad == 0, log
        r = subprocess.run([JMDEC, f"{d}/a.264", f"{d}/dec.yuv"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(f"{d}/dec.yuv", "rb").read() == open(f"{d}/a.yuv", "rb").read()


def test_rdo_changes_the_decisions():
    """RDO on and off decide differently on the same input (and both decode)."""
    ensure_built()
    cfg = ["InputFile=synthetic:81", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=16", "SymbolMode=1",
           "SearchMode=3"]
    with tempfile.TemporaryDirectory() as d:
        encode(d, cfg, "off")
        encode(d, cfg + ["RDOptimization=1"], "on")
        assert open(f"{d}/on.yuv", "rb").read() != open(f"{d}/off.yuv", "rb").read()


def test_rdo_rate_distortion_tradeoff():
    """Sanity of the Lagrangian: at the same QP the RD decisions cost fewer bits than RDO off on a
    moving sequence (both at similar quality)."""
    ensure_built()
    cfg = ["InputFile=synthetic:82", "FramesToBeEncoded=5", "ProfileIDC=77", "SearchRange=16", "SymbolMode=1",
           "SearchMode=3", "SourceWidth=352", "SourceHeight=288"]
    with tempfile.TemporaryDirectory() as d:
        off = encode(d, cfg, "off")
        on = encode(d, cfg + ["RDOptimization=1"], "on")
        bits = [int(re.search(r"bits (\d+)", x).group(1)) for x in (off, on)]
        snr = [float(re.search(r"SNR Y\(dB\) ([\d.]+)", x).group(1)) for x in (off, on)]
        assert bits[1] < bits[0], bits
        assert snr[1] > snr[0] - 0.5, snr


@pytest.mark.parametrize("bad,msg", [
    (["SearchMode=2", "ProfileIDC=77"], "SearchMode=2"),
    (["RDOptimization=2", "ProfileIDC=77"], "RDOptimization=2"),
])
def test_rdo_config_gate(bad, msg):
    ensure_built()
    with tempfile.TemporaryDirectory() as d:
        args = [LENCOD_CPU, "-p", f"OutputFile={d}/a.264", "-p", "InputFile=synthetic:1", "-p", "FramesToBeEncoded=1"]
        for e in ["SymbolMode=1", "RDOptimization=1", "SearchMode=3"] + bad:
            args += ["-p", e]
        r = subprocess.run(args, capture_output=True, text=True, timeout=60)
        assert r.returncode != 0 and msg in (r.stdout + r.stderr), r.stdout + r.stderr


def ue_bits(v):
    """length of ue(v) (9.1)"""
    return 2 * (v + 1).bit_length() - 1


@pytest.mark.parametrize("slice_mbs", [0, 11, 99])
def test_rdo_cavlc_last_mb_skip_run(slice_mbs):
    """docs/JM_SEMANTICS.md item 64(a): with CAVLC rates a P_Skip costs 0 bits (its mb_skip_run goes
    out with the next coded macroblock) except at the picture's last macroblock, where JM's
    writeMBLayer finds no next macroblock (FmoGetNextMBNr -1) and writes the pending run, this MB
    included: the skip candidate's rate is ue(run + 1).  A P picture whose source is the I
    picture's reconstruction: every macroblock is skipped."""
    import numpy as np
    import oracle_lib
    from jmpaths import load_jmhip
    ensure_built()
    jm = load_jmhip()
    w, h = 176, 144
    nmb = (w // 16) * (h // 16)
    rng = np.random.default_rng(5)
    y = rng.integers(0, 256, (h, w), dtype=np.uint8)
    u = rng.integers(0, 256, (h // 2, w // 2), dtype=np.uint8)
    v = rng.integers(0, 256, (h // 2, w // 2), dtype=np.uint8)
    o = oracle_lib.OracleEncoder(w, h, rdo=1, symbol_mode=0, search_mode=3, search_range=8, slice_mbs=slice_mbs)
    try:
        _, rec = o.encode(y, u, v, jm.JMH_I_SLICE, 28)
        o.set_reference(*rec)
        res, _ = o.encode(*rec, jm.JMH_P_SLICE, 28)       # P: its source is the reference itself
    finally:
        o.close()
    mt, mc = res["mb_type"].tolist(), res["min_cost"].tolist()
    assert mt.count(0) == nmb                              # all P_Skip
    k = slice_mbs or nmb
    run = (nmb - 1) % k                                    # skipped MBs before the last one in its slice
    assert mc[-1] == ue_bits(run + 1)
    assert all(c == 0 for c in mc[:-1])


def test_rdo_cavlc_last_mb_skip_writer():
    """the same rule through the product writer: a flat picture (its I reconstruction is exact, so
    every P macroblock is skipped, the last one included); the writer's RD rate check (the run
    written at the slice end == the last skip's rate) and the closed loop"""
    ensure_built()
    w, h, n = 96, 64, 3
    with tempfile.TemporaryDirectory() as d:
        with open(f"{d}/flat.yuv", "wb") as f:
            f.write(bytes([128]) * (w * h * 3 // 2) * n)
        log = encode(d, ["SymbolMode=0", "RDOptimization=1", "SearchMode=3", "ProfileIDC=66", "SearchRange=8",
                         f"InputFile={d}/flat.yuv", f"FramesToBeEncoded={n}", f"SourceWidth={w}", f"SourceHeight={h}"])
        nchk, bad = rate_check(log)
        assert nchk == 3 * (w // 16) * (h // 16) and bad == 0, log
        r = subprocess.run([JMDEC, f"{d}/a.264", f"{d}/dec.yuv"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(f"{d}/dec.yuv", "rb").read() == open(f"{d}/a.yuv", "rb").read()

"""Closed-loop conformance: the CPU reference encoder's bitstream, decoded by the
independent spec decoder (oracle/decoder.c), reproduces the encoder's reconstruction byte for
byte.  This pins every normative piece: CAVLC syntax, MVP, intra prediction, inverse transforms,
interpolation and the deblocking filter (two independent implementations must agree)."""
import subprocess
import tempfile

import pytest

from jmpaths import JMDEC, LENCOD_CPU, ensure_built

CONFIGS = [
    ["InputFile=synthetic:1", "FramesToBeEncoded=5", "SearchRange=16"],
    ["InputFile=synthetic:2", "FramesToBeEncoded=4", "SearchMode=-1", "SearchRange=8"],
    ["InputFile=synthetic:3", "FramesToBeEncoded=4", "UseHadamard=0"],
    ["InputFile=synthetic:4", "FramesToBeEncoded=3", "QPFirstFrame=0", "QPRemainingFrame=0", "SearchRange=4"],
    ["InputFile=synthetic:5", "FramesToBeEncoded=3", "QPFirstFrame=51", "QPRemainingFrame=51", "SearchRange=4"],
    ["InputFile=synthetic:6", "FramesToBeEncoded=6", "IntraPeriod=3", "QPFirstFrame=12", "QPRemainingFrame=20"],
    ["InputFile=synthetic:7", "FramesToBeEncoded=3", "SourceWidth=200", "SourceHeight=120", "SearchRange=8"],
    ["InputFile=synthetic:8", "FramesToBeEncoded=3", "LoopFilterParametersFlag=1", "LoopFilterAlphaC0Offset=3",
     "LoopFilterBetaOffset=-2"],
    ["InputFile=synthetic:9", "FramesToBeEncoded=3", "LoopFilterParametersFlag=1", "LoopFilterDisable=1"],
    ["InputFile=synthetic:10", "FramesToBeEncoded=3", "InterSearch16x16=0", "InterSearch8x4=0", "RestrictSearchRange=0"],
    ["InputFile=synthetic:11", "FramesToBeEncoded=3", "ChromaQPOffset=-5", "QPRemainingFrame=36"],
    ["InputFile=synthetic:12", "FramesToBeEncoded=2", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "QPRemainingFrame=40"],
    # High profile with the 8x8 transform: Intra_8x8, transform_size_8x8_flag,
    # interleaved CAVLC 8x8 residual, 8x8 deblocking edges
    ["InputFile=synthetic:21", "FramesToBeEncoded=5", "SearchRange=16", "ProfileIDC=100", "Transform8x8Mode=1"],
    ["InputFile=synthetic:22", "FramesToBeEncoded=4", "ProfileIDC=100", "Transform8x8Mode=1", "QPFirstFrame=40",
     "QPRemainingFrame=40", "SearchRange=8"],
    ["InputFile=synthetic:23", "FramesToBeEncoded=4", "ProfileIDC=100", "Transform8x8Mode=1", "QPFirstFrame=4",
     "QPRemainingFrame=8", "SearchRange=8", "UseHadamard=0"],
    ["InputFile=synthetic:24", "FramesToBeEncoded=3", "ProfileIDC=100", "Transform8x8Mode=1", "SourceWidth=200",
     "SourceHeight=120", "InterSearch8x4=0", "InterSearch4x8=0", "InterSearch4x4=0", "IntraPeriod=2",
     "QPFirstFrame=30", "QPRemainingFrame=33"],
    # EPZS (SearchMode 3), Baseline and config-3 shape (High + 8x8)
    ["InputFile=synthetic:26", "FramesToBeEncoded=5", "SearchMode=3", "SearchRange=32"],
    ["InputFile=synthetic:27", "FramesToBeEncoded=4", "SearchMode=3", "SearchRange=16", "ProfileIDC=100",
     "Transform8x8Mode=1", "SourceWidth=352", "SourceHeight=288", "QPRemainingFrame=31"],
    ["InputFile=synthetic:25", "FramesToBeEncoded=3", "ProfileIDC=100", "Transform8x8Mode=0", "SearchRange=8",
     "LoopFilterParametersFlag=1", "LoopFilterAlphaC0Offset=-2", "LoopFilterBetaOffset=3", "ChromaQPOffset=3"],
    # SliceMode 1 (row f4's slice structure): neighbours across slice edges are unavailable for
    # intra / MV prediction, CAVLC nC and the skip run; deblocking still crosses them
    ["InputFile=synthetic:31", "FramesToBeEncoded=4", "SliceMode=1", "SliceArgument=11", "SearchRange=16"],
    ["InputFile=synthetic:32", "FramesToBeEncoded=4", "SliceMode=1", "SliceArgument=7", "SearchRange=8",
     "IntraPeriod=2"],
    ["InputFile=synthetic:33", "FramesToBeEncoded=3", "SliceMode=1", "SliceArgument=1", "SearchRange=4"],
    ["InputFile=synthetic:34", "FramesToBeEncoded=3", "SliceMode=1", "SliceArgument=30", "SearchMode=-1",
     "SearchRange=8", "SourceWidth=200", "SourceHeight=120"],
    ["InputFile=synthetic:35", "FramesToBeEncoded=4", "SliceMode=1", "SliceArgument=22", "SearchMode=3",
     "SearchRange=16", "ProfileIDC=100", "Transform8x8Mode=1", "SourceWidth=352", "SourceHeight=288"],
    ["InputFile=synthetic:36", "FramesToBeEncoded=3", "SliceMode=1", "SliceArgument=13", "ProfileIDC=100",
     "Transform8x8Mode=1", "SearchMode=3", "EPZSDualRefinement=1", "QPRemainingFrame=36"],
    # SearchRange 64 (EPZS only above 32)
    ["InputFile=synthetic:37", "FramesToBeEncoded=4", "SearchMode=3", "SearchRange=64", "SourceWidth=352",
     "SourceHeight=288"],
]
# CABAC (SymbolMode 1, row f4; Main / High profile, cabac_init_idc 0): I16 / I4 / I8, P8x8 sub-partitions,
# the 8x8 transform, slices, QP extremes (levels beyond the UEG0 prefix, mvd beyond the UEG3 prefix)
CABAC = [
    ["InputFile=synthetic:41", "FramesToBeEncoded=5", "SymbolMode=1", "ProfileIDC=77", "SearchRange=16"],
    ["InputFile=synthetic:42", "FramesToBeEncoded=4", "SymbolMode=1", "ProfileIDC=77", "SearchMode=-1", "SearchRange=8",
     "IntraPeriod=2"],
    ["InputFile=synthetic:43", "FramesToBeEncoded=3", "SymbolMode=1", "ProfileIDC=77", "QPFirstFrame=0",
     "QPRemainingFrame=0", "SearchRange=4"],
    ["InputFile=synthetic:44", "FramesToBeEncoded=3", "SymbolMode=1", "ProfileIDC=77", "QPFirstFrame=51",
     "QPRemainingFrame=51", "SearchRange=4"],
    ["InputFile=synthetic:45", "FramesToBeEncoded=5", "SymbolMode=1", "ProfileIDC=100", "Transform8x8Mode=1",
     "SearchRange=16"],
    ["InputFile=synthetic:46", "FramesToBeEncoded=4", "SymbolMode=1", "ProfileIDC=100", "Transform8x8Mode=1",
     "QPFirstFrame=4", "QPRemainingFrame=8", "SearchRange=8", "UseHadamard=0"],
    ["InputFile=synthetic:47", "FramesToBeEncoded=4", "SymbolMode=1", "ProfileIDC=77", "SliceMode=1",
     "SliceArgument=11", "SearchRange=16", "ChromaQPOffset=-5", "QPRemainingFrame=36"],
    ["InputFile=synthetic:48", "FramesToBeEncoded=4", "SymbolMode=1", "ProfileIDC=100", "Transform8x8Mode=1",
     "SearchMode=3", "SearchRange=16", "SourceWidth=352", "SourceHeight=288", "SliceMode=1", "SliceArgument=22",
     "QPRemainingFrame=31"],
    ["InputFile=synthetic:49", "FramesToBeEncoded=3", "SymbolMode=1", "ProfileIDC=77", "SliceMode=1",
     "SliceArgument=1", "SearchRange=8", "SourceWidth=200", "SourceHeight=120"],
    ["InputFile=synthetic:50", "FramesToBeEncoded=3", "SymbolMode=1", "ProfileIDC=100", "Transform8x8Mode=1",
     "InterSearch16x16=0", "InterSearch8x4=0", "RestrictSearchRange=0", "LoopFilterParametersFlag=1",
     "LoopFilterAlphaC0Offset=3", "LoopFilterBetaOffset=-2", "QPFirstFrame=12", "QPRemainingFrame=20"],
]

# High 10 (ProfileIDC 110): 9 / 10-bit samples through EPZS, I4 / I16 / I8, the 8x8
# transform, QP'Y / QP'C = QP + 6 (bit depth - 8) (incl. negative QPc), scaled deblocking thresholds,
# CAVLC and CABAC, slices, QP extremes
HIGH10 = [
    ["InputFile=synthetic:61", "FramesToBeEncoded=4", "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10",
     "SearchMode=3", "SearchRange=16"],
    ["InputFile=synthetic:62", "FramesToBeEncoded=4", "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10",
     "SearchMode=3", "SearchRange=16", "Transform8x8Mode=1", "SourceWidth=352", "SourceHeight=288", "QPRemainingFrame=31"],
    ["InputFile=synthetic:63", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=9", "SourceBitDepthChroma=9",
     "SearchMode=3", "SearchRange=8", "Transform8x8Mode=1", "QPFirstFrame=0", "QPRemainingFrame=2", "ChromaQPOffset=-12"],
    ["InputFile=synthetic:64", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10",
     "SearchMode=3", "SearchRange=8", "QPFirstFrame=51", "QPRemainingFrame=51", "LoopFilterParametersFlag=1",
     "LoopFilterAlphaC0Offset=6", "LoopFilterBetaOffset=6"],
    ["InputFile=synthetic:65", "FramesToBeEncoded=4", "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10",
     "SearchMode=3", "SearchRange=16", "Transform8x8Mode=1", "SymbolMode=1", "SliceMode=1", "SliceArgument=13",
     "EPZSDualRefinement=1", "IntraPeriod=2"],
    ["InputFile=synthetic:66", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10",
     "SearchMode=3", "SearchRange=8", "SymbolMode=1", "QPFirstFrame=4", "QPRemainingFrame=6", "UseHadamard=0",
     "SourceWidth=200", "SourceHeight=120"],
    # FFS and full search on 16-bit samples
    ["InputFile=synthetic:67", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10",
     "SearchMode=0", "SearchRange=16", "Transform8x8Mode=1"],
    ["InputFile=synthetic:68", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=9", "SourceBitDepthChroma=9",
     "SearchMode=-1", "SearchRange=8", "RestrictSearchRange=0", "SymbolMode=1", "QPFirstFrame=10", "QPRemainingFrame=12"],
]

# UseConstrainedIntraPred 1 (constrained_intra_pred_flag): intra MBs of P pictures predict only
# from intra neighbours (inter neighbours' samples "not available for Intra prediction", 8.3), and
# an inter neighbour sets dcPredModePredictedFlag (8.3.1.1); CAVLC / CABAC, I4 / I8 / I16, slices, RDO
CIP = [
    ["InputFile=synthetic:81", "FramesToBeEncoded=5", "SearchRange=2", "QPRemainingFrame=20", "UseConstrainedIntraPred=1"],
    ["InputFile=synthetic:82", "FramesToBeEncoded=4", "UseConstrainedIntraPred=1", "SymbolMode=1", "ProfileIDC=77",
     "QPRemainingFrame=40", "SearchRange=8"],
    ["InputFile=synthetic:83", "FramesToBeEncoded=4", "UseConstrainedIntraPred=1", "ProfileIDC=100", "Transform8x8Mode=1",
     "SearchMode=3", "SearchRange=4", "SliceMode=1", "SliceArgument=13", "QPRemainingFrame=24"],
    ["InputFile=synthetic:84", "FramesToBeEncoded=3", "UseConstrainedIntraPred=1", "RDOptimization=1", "SymbolMode=1",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3", "SearchRange=8", "QPRemainingFrame=30"],
    ["InputFile=synthetic:85", "FramesToBeEncoded=3", "UseConstrainedIntraPred=1", "ProfileIDC=110", "SourceBitDepthLuma=10",
     "SourceBitDepthChroma=10", "SearchMode=3", "SearchRange=8", "RDOptimization=1", "QPRemainingFrame=44"],
]


def encode(d, extra):
    args = [LENCOD_CPU, "-p", f"OutputFile={d}/a.264", "-p", f"ReconFile={d}/rec.yuv"]
    for e in extra:
        args += ["-p", e]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("extra", CONFIGS, ids=[c[0].split(":")[1] for c in CONFIGS])
def test_decoder_reproduces_recon(extra):
    ensure_built()
    with tempfile.TemporaryDirectory() as d:
        encode(d, extra)
        r = subprocess.run([JMDEC, f"{d}/a.264", f"{d}/dec.yuv"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(f"{d}/dec.yuv", "rb").read() == open(f"{d}/rec.yuv", "rb").read()


@pytest.mark.parametrize("extra", CABAC, ids=[c[0].split(":")[1] for c in CABAC])
def test_decoder_reproduces_recon_cabac(extra):
    """SymbolMode 1: the independent decoder's CABAC parser (own tables and context selection)
    reproduces the encoder's reconstruction."""
    test_decoder_reproduces_recon(extra)


@pytest.mark.parametrize("extra", HIGH10, ids=[c[0].split(":")[1] for c in HIGH10])
def test_decoder_reproduces_recon_high10(extra):
    """High 10: the decoder's 16-bit path reproduces the encoder's 16-bit reconstruction."""
    test_decoder_reproduces_recon(extra)


def test_high10_recon_uses_the_range():
    """10-bit reconstruction: 16-bit LE samples, some above 255 (not an 8-bit picture stored wide)."""
    ensure_built()
    import numpy as np
    with tempfile.TemporaryDirectory() as d:
        encode(d, HIGH10[0])
        rec = np.fromfile(f"{d}/rec.yuv", "<u2")
        assert rec.max() > 255 and rec.max() <= 1023


def test_cabac_smaller_than_cavlc():
    """The same decisions coded with CABAC take fewer bits than with CAVLC (same recon)."""
    ensure_built()
    with tempfile.TemporaryDirectory() as a, tempfile.TemporaryDirectory() as b:
        base = ["InputFile=synthetic:51", "FramesToBeEncoded=4", "ProfileIDC=77", "SearchRange=16"]
        encode(a, base)
        encode(b, base + ["SymbolMode=1"])
        assert open(f"{a}/rec.yuv", "rb").read() == open(f"{b}/rec.yuv", "rb").read()
        va, vb = len(open(f"{a}/a.264", "rb").read()), len(open(f"{b}/a.264", "rb").read())
        assert vb < va, (va, vb)


def test_deterministic_bitstream():
    ensure_built()
    with tempfile.TemporaryDirectory() as a, tempfile.TemporaryDirectory() as b:
        encode(a, CONFIGS[0])
        encode(b, CONFIGS[0])
        assert open(f"{a}/a.264", "rb").read() == open(f"{b}/a.264", "rb").read()


def nal_types(buf):
    """NAL unit types of an Annex B byte stream"""
    out, i = [], 0
    while i + 3 < len(buf):
        if buf[i] == 0 and buf[i + 1] == 0 and buf[i + 2] == 1:
            out.append(buf[i + 3] & 31)
            i += 3
        else:
            i += 1
    return out


@pytest.mark.parametrize("arg,nslices", [(11, 9), (7, 15), (99, 1), (500, 1)])
def test_slice_count(arg, nslices):
    """SliceMode 1: ceil(99 / SliceArgument) slice NAL units per QCIF picture, first_mb_in_slice
    advancing by SliceArgument; the decoder reassembles each picture from its slices."""
    ensure_built()
    with tempfile.TemporaryDirectory() as d:
        encode(d, ["InputFile=synthetic:37", "FramesToBeEncoded=3", "SliceMode=1", f"SliceArgument={arg}",
                   "SearchRange=8"])
        t = nal_types(open(f"{d}/a.264", "rb").read())
        assert t.count(5) == nslices and t.count(1) == 2 * nslices
        r = subprocess.run([JMDEC, f"{d}/a.264", f"{d}/dec.yuv"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(f"{d}/dec.yuv", "rb").read() == open(f"{d}/rec.yuv", "rb").read()


def test_slices_change_the_decisions():
    """Slice edges remove neighbours: one MB per slice differs from one slice per picture."""
    ensure_built()
    with tempfile.TemporaryDirectory() as a, tempfile.TemporaryDirectory() as b:
        base = ["InputFile=synthetic:38", "FramesToBeEncoded=2", "SearchRange=8"]
        encode(a, base)
        encode(b, base + ["SliceMode=1", "SliceArgument=1"])
        assert open(f"{a}/rec.yuv", "rb").read() != open(f"{b}/rec.yuv", "rb").read()


@pytest.mark.parametrize("arg", [1, 5, 99])
def test_slices_of_skipped_macroblocks(arg):
    """A still picture repeated: P slices that are (almost) all P_Skip, so slices end on a trailing
    mb_skip_run (or consist of one); the decoder's more_rbsp_data() must end each slice there."""
    ensure_built()
    import numpy as np
    rng = np.random.default_rng(arg)
    y = rng.integers(0, 256, (144, 176), dtype=np.uint8)
    y = ((y.astype(np.uint16) + np.roll(y, 1, 0) + np.roll(y, 1, 1)) // 3).astype(np.uint8)
    frame = y.tobytes() + y[::2, ::2].tobytes() + y[1::2, 1::2].tobytes()
    with tempfile.TemporaryDirectory() as d:
        with open(f"{d}/in.yuv", "wb") as f:
            f.write(frame * 3)
        encode(d, [f"InputFile={d}/in.yuv", "FramesToBeEncoded=3", "SliceMode=1", f"SliceArgument={arg}",
                   "SearchRange=8", "QPFirstFrame=20", "QPRemainingFrame=30"])
        r = subprocess.run([JMDEC, f"{d}/a.264", f"{d}/dec.yuv"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(f"{d}/dec.yuv", "rb").read() == open(f"{d}/rec.yuv", "rb").read()
        assert len(nal_types(open(f"{d}/a.264", "rb").read())) == 2 + 3 * -(-99 // arg)


@pytest.mark.parametrize("extra", CIP, ids=[c[0].split(":")[1] for c in CIP])
def test_decoder_reproduces_recon_constrained_intra(extra):
    """UseConstrainedIntraPred 1: the decoder's constrained intra availability and mode prediction
    reproduce the encoder's reconstruction -- and the flag changes it (intra MBs next to inter ones)."""
    test_decoder_reproduces_recon(extra)
    with tempfile.TemporaryDirectory() as d, tempfile.TemporaryDirectory() as d0:
        encode(d, extra)
        encode(d0, [e for e in extra if not e.startswith("UseConstrainedIntraPred")])
        assert open(f"{d}/rec.yuv", "rb").read() != open(f"{d0}/rec.yuv", "rb").read()

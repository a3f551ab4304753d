"""JM >= 10 EPZS as shipped (row a15, docs/JM_SEMANTICS.md items 61, 62): the neighbour-adaptive
stop criterion (EPZSMinThresScale / EPZSMaxThresScale, EPZSDetermineStopCriterion) and the EPZS
sub-pel pattern search (EPZSSubPelME, EPZSSubPelThresScale).

CPU: lencod_cpu's closed loop through the independent decoder with each knob and with the
JM >= 10 encoder.cfg combination, that each knob changes the bitstream, a property of the sub-pel
stages (with the quarter stage always skipped every MV is the full-pel MV plus a half-pel
offset: even), and the knob ranges.  GPU: whole pictures == the oracle bit for bit (RDO off and
on, 8 and 10 bits, slices, SATD / SAD).  JM parity is unpinned (no JM source in the reference):
these restate JM >= 10's options from their published description."""
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib
from jmpaths import JMDEC, LENCOD_CPU, ensure_built, load_jmhip

jmhip = load_jmhip()

# the JM >= 10 encoder.cfg EPZS block as this build restates it
JM10_EPZS = ["EPZSSubPelME=1", "EPZSSubPelThresScale=2", "EPZSMinThresScale=0", "EPZSMaxThresScale=2", "EPZSDualRefinement=1"]
CASES = [
    ["InputFile=synthetic:81", "FramesToBeEncoded=4", "SearchMode=3", "SearchRange=32", "EPZSSubPelME=1"],
    ["InputFile=synthetic:82", "FramesToBeEncoded=4", "SearchMode=3", "SearchRange=32", "EPZSMaxThresScale=8",
     "EPZSMinThresScale=4"],
    ["InputFile=synthetic:83", "FramesToBeEncoded=4", "SearchMode=3", "SearchRange=16", "ProfileIDC=100",
     "Transform8x8Mode=1", "JMVersion=10", "QPRemainingFrame=30"] + JM10_EPZS,
    ["InputFile=synthetic:84", "FramesToBeEncoded=3", "SearchMode=3", "SearchRange=16", "UseHadamard=0",
     "SliceMode=1", "SliceArgument=13"] + JM10_EPZS,
    ["InputFile=synthetic:85", "FramesToBeEncoded=3", "SearchMode=3", "SearchRange=16", "ProfileIDC=110",
     "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "SymbolMode=1", "RDOptimization=1"] + JM10_EPZS,
]
IDS = ["subpel", "thres", "high-jm10", "sad-slices", "high10-rdo"]
KNOBS = ("EPZSSubPelME", "EPZSSubPelThresScale", "EPZSMinThresScale", "EPZSMaxThresScale", "EPZSDualRefinement")


def run(*args):
    ensure_built()
    return subprocess.run([LENCOD_CPU, *args], capture_output=True, text=True, timeout=300)


def encode(d, extra, name="a"):
    args = ["-p", f"OutputFile={d}/{name}.264", "-p", f"ReconFile={d}/{name}.yuv"]
    for e in extra:
        args += ["-p", e]
    r = run(*args)
    assert r.returncode == 0, r.stdout + r.stderr
    return open(f"{d}/{name}.264", "rb").read()


# ---------------- CPU ----------------
@pytest.mark.parametrize("extra", CASES, ids=IDS)
def test_closed_loop_epzs_jm10(extra):
    with tempfile.TemporaryDirectory() as d:
        bs = encode(d, extra)
        r = subprocess.run([JMDEC, f"{d}/a.264", f"{d}/dec.yuv"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert open(f"{d}/dec.yuv", "rb").read() == open(f"{d}/a.yuv", "rb").read()
        plain = [e for e in extra if not e.startswith(KNOBS)]
        assert encode(d, plain, "b") != bs, "the EPZS options did not change the bitstream"


def test_quarter_stage_skipped_gives_half_pel_mvs():
    """EPZSSubPelThresScale at its maximum skips the quarter-pel stage of (almost) every search, so
    every MV is the full-pel MV plus a half-pel offset; with the threshold 0 quarter-pel MVs occur."""
    w, h = 176, 144
    pics = [jmhip.synth_frame(w, h, 86, i) for i in range(3)]
    odd = []
    for scale in (63, 0):
        o = oracle_lib.OracleEncoder(w, h, search_range=16, search_mode=3, epzs_subpel_me=1, epzs_subpel_thres_scale=scale)
        n = 0
        for i, pic in enumerate(pics):
            res, rec = o.encode(*pic, jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE, 28)
            inter = (res["mb_type"] >= 1) & (res["mb_type"] <= 8)
            n += int((res["mv"][inter] & 1).sum())
            o.set_reference(*rec)
        odd.append(n)
    assert odd[0] == 0 and odd[1] > 0, odd


def test_epzs_knob_ranges():
    for bad in ("EPZSSubPelME=2", "EPZSMaxThresScale=64", "EPZSSubPelThresScale=64", "EPZSMinThresScale=-1"):
        r = run("-p", "SearchMode=3", "-p", bad)
        assert r.returncode != 0 and bad.split("=")[0] in r.stderr, bad
    for kw in (dict(epzs_subpel_me=2), dict(epzs_max_thres_scale=64), dict(epzs_subpel_thres_scale=-1)):
        with pytest.raises(Exception):
            oracle_lib.OracleEncoder(64, 48, search_range=8, search_mode=3, **kw)


# ---------------- GPU ----------------
GPU_CASES = [
    (dict(search_range=32, epzs_subpel_me=1), 28),
    (dict(search_range=32, epzs_max_thres_scale=8, epzs_min_thres_scale=4), 28),
    (dict(search_range=32, epzs_subpel_me=1, epzs_subpel_thres_scale=2, epzs_max_thres_scale=2, epzs_dual_refinement=1), 24),
    (dict(search_range=16, use_hadamard=0, epzs_subpel_me=1, epzs_subpel_thres_scale=63, epzs_max_thres_scale=1), 33),
    (dict(search_range=16, transform_8x8_mode=1, jm_version=10, slice_mbs=13, epzs_subpel_me=1, epzs_subpel_thres_scale=2,
          epzs_max_thres_scale=2, epzs_dual_refinement=1), 30),
    (dict(search_range=16, inter_search=(1, 0, 0, 1, 0, 1, 1), epzs_subpel_me=1, epzs_max_thres_scale=3, epzs_min_thres_scale=2), 26),
]


@pytest.mark.gpu
@pytest.mark.parametrize("kw,qp", GPU_CASES)
def test_gpu_epzs_jm10(kw, qp):
    from test_gpu_parity import encode_pair, moving_seq, shear_seq
    for pics in (moving_seq(176, 144, 4, seed=91, step=(13, -7)), shear_seq(176, 144, 4, seed=92)):
        encode_pair(176, 144, pics, [jmhip.JMH_I_SLICE] + [jmhip.JMH_P_SLICE] * 3, qp, search_mode=3, **kw)


@pytest.mark.gpu
@pytest.mark.parametrize("bd,rdo", [(10, 0), (10, 1), (8, 1)])
def test_gpu_epzs_jm10_high10_rdo(bd, rdo):
    from test_gpu_parity import encode_pair, hbd_seq, moving_seq
    kw = dict(search_range=16, search_mode=3, epzs_subpel_me=1, epzs_subpel_thres_scale=2, epzs_max_thres_scale=2,
              epzs_dual_refinement=1, slice_mbs=11, bit_depth=bd)
    if rdo:
        kw.update(rdo=1, symbol_mode=1)
    pics = hbd_seq(176, 144, 3, seed=93, bd=bd) if bd > 8 else moving_seq(176, 144, 3, seed=93, step=(9, 5))
    encode_pair(176, 144, pics, [jmhip.JMH_I_SLICE] + [jmhip.JMH_P_SLICE] * 2, 29, **kw)


@pytest.mark.gpu
def test_gpu_epzs_jm10_3840():
    """The 3840-wide shape (config 3 / 5 width) with the JM >= 10 EPZS options."""
    from test_gpu_parity import encode_pair, hbd_seq
    pics = hbd_seq(3840, 96, 3, seed=94, bd=10)
    encode_pair(3840, 96, pics, [jmhip.JMH_I_SLICE] + [jmhip.JMH_P_SLICE] * 2, 28, search_mode=3, search_range=32, bit_depth=10,
                slice_mbs=240, epzs_subpel_me=1, epzs_subpel_thres_scale=2, epzs_max_thres_scale=2, epzs_dual_refinement=1)

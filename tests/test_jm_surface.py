"""The JM 8.6 call surface (host/jm86.c, SURVEY.md §8b "what the build keeps"): lencod's slice
loop calls start_macroblock → encode_one_macroblock → write_one_macroblock per macroblock, and
encode_one_macroblock can run JM's RDO-off inter searches through PartitionMotionSearch →
BlockMotionSearch (one device search per call, jmh_block_motion_search) and check the wavefront
decision against them.  dct_luma runs one block through jmh_tq4x4_batch.

CPU tests drive the same host code over the oracle backend (lencod_cpu); GPU tests drive it
over libjmhip.so and compare with the oracle call by call.
"""
import ctypes
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib
from jmpaths import JM86_CHECK, LENCOD, LENCOD_CPU, ensure_built, load_jmhip

jmhip = load_jmhip()

CASES = [
    ["InputFile=synthetic:1", "FramesToBeEncoded=3", "SourceWidth=176", "SourceHeight=144", "SearchRange=16"],
    ["InputFile=synthetic:7", "FramesToBeEncoded=3", "SourceWidth=176", "SourceHeight=144", "SearchRange=8",
     "SearchMode=-1", "RestrictSearchRange=0"],
    ["InputFile=synthetic:9", "FramesToBeEncoded=2", "SourceWidth=208", "SourceHeight=112", "SearchRange=12",
     "RestrictSearchRange=1", "UseHadamard=0", "QPRemainingFrame=36", "InterSearch8x4=0"],
    # SliceMode 1: SetMotionVectorPredictor sees only the current slice (img->slice_first)
    ["InputFile=synthetic:11", "FramesToBeEncoded=3", "SourceWidth=176", "SourceHeight=144", "SearchRange=8",
     "SliceMode=1", "SliceArgument=8"],
]


def run(binary, out, extra, surface):
    args = [binary, "-p", f"OutputFile={out}", "-p", f"JMCallSurface={surface}"]
    for e in extra:
        args += ["-p", e]
    r = subprocess.run(args, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.parametrize("extra", CASES)
def test_cpu_call_surface_reproduces_the_decisions(extra):
    """CPU build: JM-ordered PartitionMotionSearch / BlockMotionSearch calls per P macroblock
    agree with every decision, and the slice loop writes the same bitstream either way."""
    ensure_built()
    with tempfile.TemporaryDirectory() as d:
        log = run(LENCOD_CPU, f"{d}/s.264", extra, 1)
        run(LENCOD_CPU, f"{d}/p.264", extra, 0)
        assert " 0 inconsistent" in log and "JM call surface: 0 P" not in log, log
        assert open(f"{d}/s.264", "rb").read() == open(f"{d}/p.264", "rb").read()


def block_requests(w, h, sr, n, seed):
    rng = np.random.default_rng(seed)
    bsz = {1: (4, 4), 2: (4, 2), 3: (2, 4), 4: (2, 2), 5: (2, 1), 6: (1, 2), 7: (1, 1)}
    reqs = (jmhip.JmhBlockSearch * n)()
    for q in reqs:
        bt = int(rng.integers(1, 8))
        bw, bh = bsz[bt]
        q.mb_x, q.mb_y = int(rng.integers(0, w // 16)), int(rng.integers(0, h // 16))
        q.blocktype = bt
        q.block_x, q.block_y = int(rng.integers(0, 5 - bw)) // bw * bw, int(rng.integers(0, 5 - bh)) // bh * bh
        q.pred_mv[0], q.pred_mv[1] = (int(v) for v in rng.integers(-4 * sr - 40, 4 * sr + 40, 2))
        q.search_range = int(rng.integers(0, sr + 1))
        q.search_mode = int(rng.choice([0, -1]))
        if q.search_mode == 0:
            q.centre[0], q.centre[1] = (int(v) for v in rng.integers(-sr, sr + 1, 2))
        else:
            q.centre[0] = max(-q.search_range, min(q.search_range, int(q.pred_mv[0] / 4)))
            q.centre[1] = max(-q.search_range, min(q.search_range, int(q.pred_mv[1] / 4)))
        q.lambda_factor = int(65536 * rng.choice([1, 4, 25, 91]) + (0 if rng.random() < 0.7 else rng.integers(0, 65536)))
        q.slice_p = int(rng.random() < 0.9)
    return reqs


@pytest.mark.gpu
@pytest.mark.parametrize("had", [1, 0])
def test_block_motion_search_seam(had):
    """jmh_block_motion_search == the oracle's BlockMotionSearch on random requests (all block
    types, FFS and full search, restricted ranges, non-integer lambda factors, edge MBs)."""
    w, h, sr = 176, 144, 16
    pics = [jmhip.synth_frame(w, h, 4, i) for i in range(2)]
    g = jmhip.Encoder(w, h, search_range=sr, use_hadamard=had)
    o = oracle_lib.OracleEncoder(w, h, search_range=sr, use_hadamard=had)
    g.search_pictures(pics[1][0], pics[0][0])
    o.search_pictures(pics[1][0], pics[0][0])
    reqs = block_requests(w, h, sr, 300, 11 + had)
    gr, orr = g.block_motion_search(reqs), o.block_motion_search(reqs)
    for i, (a, b) in enumerate(zip(gr, orr)):
        assert bytes(a) == bytes(b), (i, list(a.mv), a.min_mcost, list(b.mv), b.min_mcost)
    g.close()


@pytest.mark.gpu
def test_jm86_check_binary():
    """dct_luma on every QP and BlockMotionSearch through encode_one_macroblock, device vs
    oracle, call by call (oracle/jm86_check.c)."""
    ensure_built()
    r = subprocess.run([JM86_CHECK], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout and "0 decisions inconsistent" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("extra", CASES)
def test_lencod_call_surface(extra):
    """GPU lencod with JMCallSurface=1: every P macroblock's JM-ordered device searches agree
    with the wavefront decision; the bitstream equals the default loop's and the CPU build's."""
    with tempfile.TemporaryDirectory() as d:
        log = run(LENCOD, f"{d}/s.264", extra, 1)
        run(LENCOD, f"{d}/p.264", extra, 0)
        run(LENCOD_CPU, f"{d}/c.264", extra, 0)
        assert " 0 inconsistent" in log and "JM call surface: 0 P" not in log, log
        s = open(f"{d}/s.264", "rb").read()
        assert s == open(f"{d}/p.264", "rb").read() == open(f"{d}/c.264", "rb").read()

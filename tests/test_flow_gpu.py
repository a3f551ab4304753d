"""The dataflow wavefront (k_mb_flow) == the tick wavefront, bit for bit.

With SearchMode 0 on 8-bit samples and RDO off the library collects a segment of ticks and runs
it as one launch of one workgroup per macroblock, each waiting on per-MB flags for the macroblocks
it depends on.  These tests run the same chains with JMH_FLOW=0 (one k_mb_analyse + k_mb_final
launch per tick, the path every earlier round measured) and compare every result field, the
reconstruction and the deblocked reference; segment lengths from one tick to the default stress the
flush points (readback, entry reuse, drains).  The oracle comparisons of test_gpu_parity.py run
through the dataflow path by default.
"""
import os

import numpy as np
import pytest

from jmpaths import ensure_built, load_jmhip
from test_gpu_parity import assert_same, moving_seq, run_chain

jmhip = load_jmhip()
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def built():
    ensure_built()
    jmhip.load()


class env:
    """Environment knobs read by jmh_create (set around the Encoder's construction)."""

    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def chain(w, h, sr, pics, pipelined=True, qp=30, **kw):
    enc = jmhip.Encoder(w, h, search_range=sr, **kw)
    out = run_chain(enc, pics, qp, (0, 0, 0), pipelined)
    enc.close()
    return out


def same_chains(ra, rb, w):
    assert len(ra) == len(rb)
    for (gres, grec, gdbk), (ores, orec, odbk) in zip(ra, rb):
        assert_same(gres, grec, ores, orec, w // 16)
        for x, y in zip(gdbk, odbk):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("w,h,sr,n,step,seg,kw", [
    (176, 144, 16, 9, (37, -29), None, {}),
    (1920, 1088, 32, 12, (37, -29), None, {}),
    (1920, 1088, 32, 10, (-62, -61), 1, {}),          # every tick its own launch
    (1920, 1088, 32, 10, (63, 62), 7, {}),
    (256, 4096, 32, 36, (37, -29), None, {}),           # 526 diagonals, ~33 pictures in flight
    (1920, 1088, 32, 10, (37, -29), 5, dict(slice_mbs=120)),
    (640, 480, 32, 10, (-62, -61), None, dict(slice_mbs=57, restrict_search_range=0)),
])
def test_flow_equals_ticks(w, h, sr, n, step, seg, kw):
    """Pipelined push / pop chains, MVs up to the search-window edge: dataflow == ticks."""
    pics = moving_seq(w, h, n, seed=w + 3 * n, step=step)
    with env(JMH_FLOW=0):
        rt = chain(w, h, sr, pics, **kw)
    with env(JMH_FLOW=1, **({"JMH_FLOW_SEG": seg} if seg else {})):
        rf = chain(w, h, sr, pics, **kw)
    same_chains(rf, rt, w)
    assert any((r["mb_type"] != 0).any() for r, _, _ in rf[1:])


def test_flow_sequential_equals_ticks():
    """One picture at a time (pipeline depth 1: every picture its own segment)."""
    w, h = 352, 288
    pics = moving_seq(w, h, 6, seed=11, step=(-21, 13))
    with env(JMH_FLOW=0):
        rt = chain(w, h, 32, pics, pipelined=False, pipeline_depth=1)
    with env(JMH_FLOW=1):
        rf = chain(w, h, 32, pics, pipelined=False, pipeline_depth=1)
    same_chains(rf, rt, w)


@pytest.mark.parametrize("seg", [None, 3])
def test_flow_slots_long_chain(seg):
    """bench.py's path: a long encode_slot chain without readback (segments of many ticks, ring
    entries reused inside them, the device head counter carried across launches), then a read-back
    picture: equal to the tick path."""
    w, h = 352, 288
    pics = moving_seq(w, h, 4, seed=5, step=(-21, 13))
    res = []
    for flow in (0, 1):
        with env(JMH_FLOW=flow, **({"JMH_FLOW_SEG": seg} if seg else {})):
            e = jmhip.Encoder(w, h, search_range=32, slots=3)
        for i in range(3):
            e.load_frame(i, *pics[i])
        e.encode_slot(0, jmhip.JMH_I_SLICE, 28, deblock=(0, 0, 0))
        for k in range(70):
            e.set_reference_slot(-2)
            e.encode_slot(1 + k % 2, jmhip.JMH_P_SLICE, 28, deblock=(0, 0, 0))
        e.set_reference_slot(-2)
        res.append(e.encode(*pics[3], jmhip.JMH_P_SLICE, 28, deblock=(0, 0, 0)) + (e.deblocked(),))
        t = e.timing()
        if flow:
            assert t.flow_launches > 0 and t.flow_mbs > 0
        else:
            assert t.flow_launches == 0
        e.close()
    (gres, grec, gd), (ores, orec, od) = res
    assert_same(gres, grec, ores, orec, w // 16)
    for x, y in zip(gd, od):
        assert np.array_equal(x, y)


def test_flow_intra_period():
    """I pictures inside the chain (intra_role on the dataflow path) and the reference switching
    back to the I picture's deblocking."""
    w, h = 320, 240
    pics = moving_seq(w, h, 8, seed=21, step=(29, -23))
    outs = []
    for flow in (0, 1):
        with env(JMH_FLOW=flow):
            enc = jmhip.Encoder(w, h, search_range=16)
        out = []
        pending = 0
        for i, pic in enumerate(pics):
            st = jmhip.JMH_I_SLICE if i % 3 == 0 else jmhip.JMH_P_SLICE
            if st == jmhip.JMH_P_SLICE:
                enc.set_reference_slot(-2)
            if pending == enc.depth:
                out.append(enc.pop() + (enc.deblocked(),))
                pending -= 1
            enc.push(*pic, st, 26, deblock=(0, 0, 0))
            pending += 1
        for _ in range(pending):
            out.append(enc.pop() + (enc.deblocked(),))
        enc.close()
        outs.append(out)
    same_chains(outs[1], outs[0], w)

"""Config 4's execution model on the device: `bench.py --gpus 2` launches two ranks (one process
each, gloo for the timing reduction only), each encoding its own HIP stream (seed = rank).  On
the one-GPU test box both ranks share device 0; on an 8-GPU node rank k runs on device k.

Each rank dumps one read-back picture after its timed chain (it depends on every picture of the
chain through the reference).  It must equal (a) the same chain encoded undistributed and one
picture at a time in this process and (b) the oracle's chain for that seed, bit for bit.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib
from jmpaths import ROOT, ensure_built, load_jmhip

jmhip = load_jmhip()
W, H, SR, QP = 352, 288, 32, 28


def chain_frames(seed, nframes):
    return [jmhip.synth_frame(W, H, seed, i) for i in range(nframes + 1)]


def replay(enc, frames, slots):
    """I picture, the P chain in the order the rank ran it (each referencing the previous
    reconstruction, no loop filter), then the read-back picture frames[1]."""
    enc.encode(*frames[0], jmhip.JMH_I_SLICE, QP)
    for s in list(slots) + [1]:
        rec = enc.recon()
        enc.set_reference(*rec)
        res, rec = enc.encode(*frames[s], jmhip.JMH_P_SLICE, QP)
    return res, rec


class OracleReplay(oracle_lib.OracleEncoder):
    def encode(self, *a, **k):
        self._last = super().encode(*a, **k)
        return self._last

    def recon(self):
        return self._last[1]


@pytest.mark.gpu
def test_two_hip_streams_as_two_processes(tmp_path):
    ensure_built()
    nframes, steps = 3, 3
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", str(steps), "--warmup", "2",
           "--frames", str(nframes), "--size", f"{W}x{H}", "--no-cpu-baseline", "--no-deblock", "--dump", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["timed_region"]["pictures_completed"] == [steps, steps]
    digests = []
    for rank in range(2):
        d = np.load(tmp_path / f"rank{rank}.npz")
        assert len(d["slots"]) == int(d["warmup"]) + steps
        frames = chain_frames(rank, nframes)
        g = jmhip.Encoder(W, H, search_range=SR, pipeline_depth=1)
        gres, grec = replay(g, frames, d["slots"])
        g.close()
        o = OracleReplay(W, H, search_range=SR)
        ores, orec = replay(o, frames, d["slots"])
        o.close()
        for ref_res, ref_rec in ((gres, grec), (ores, orec)):
            assert d["res"].tobytes() == ref_res.tobytes()
            for k, plane in zip("yuv", ref_rec):
                assert np.array_equal(d[k], plane)
        digests.append(d["res"].tobytes())
    assert digests[0] != digests[1]            # distinct seeds -> distinct streams


@pytest.mark.gpu
def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr

"""Golden fixtures (tests/golden/, made by tools/make_golden.py): the oracle must keep producing
them (CPU), and the MI355X path must produce the same stored outputs (GPU) — bitstream and
reconstruction digests of lencod runs, per-picture macroblock results of an I-P-P sequence, and
the dct_luma / quarter-pel / FFS SAD-table unit vectors.
"""
import hashlib
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_lib
from jmpaths import LENCOD, LENCOD_CPU, ROOT, ensure_built, load_jmhip

GOLD = os.path.join(ROOT, "tests", "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))
jmhip = load_jmhip()


def sha(b):
    return hashlib.sha256(b).hexdigest()


def npz(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def lencod_digests(binary, params):
    with tempfile.TemporaryDirectory() as d:
        args = [binary, "-p", f"OutputFile={d}/a.264", "-p", f"ReconFile={d}/rec.yuv"]
        for p in params:
            args += ["-p", p]
        r = subprocess.run(args, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stdout + r.stderr
        return sha(open(f"{d}/a.264", "rb").read()), sha(open(f"{d}/rec.yuv", "rb").read())


def sequence(encode_factory):
    spec = MANIFEST["sequence"]["spec"]
    enc = encode_factory(spec["w"], spec["h"], spec["search_range"])
    got = []
    for i in range(spec["frames"]):
        pic = jmhip.synth_frame(spec["w"], spec["h"], spec["seed"], i)
        res, rec = enc.encode(*pic, jmhip.JMH_I_SLICE if i == 0 else jmhip.JMH_P_SLICE, spec["qp"])
        enc.set_reference(*rec)
        got.append({"results": sha(res.tobytes()), "recon": sha(b"".join(p.tobytes() for p in rec))})
    return got


# ---------------- oracle (CPU) ----------------
@pytest.fixture(scope="module", autouse=True)
def built():
    ensure_built()


@pytest.mark.parametrize("case", range(len(MANIFEST["lencod"])))
def test_oracle_lencod_matches_golden(case):
    g = MANIFEST["lencod"][case]
    assert lencod_digests(LENCOD_CPU, g["params"]) == (g["bitstream_sha256"], g["recon_sha256"])


def test_oracle_sequence_matches_golden():
    assert sequence(lambda w, h, sr: oracle_lib.OracleEncoder(w, h, search_range=sr)) == MANIFEST["sequence"]["pictures"]


def test_oracle_tq4x4_matches_golden():
    z = npz("tq4x4.npz")
    for qp in (0, 12, 28, 51):
        for intra in (0, 1):
            got = oracle_lib.tq4x4(z["resid"], z["pred"], qp, intra)
            for name, arr in zip(("lev", "rec", "cc", "nz"), got):
                assert np.array_equal(arr, z[f"{name}_{qp}_{intra}"]), (name, qp, intra)


def test_oracle_qpel_matches_golden():
    z = npz("qpel.npz")
    h, w = z["y"].shape
    o = oracle_lib.OracleEncoder(w, h, search_range=4)
    o.set_reference(z["y"], z["u"], z["v"])
    assert np.array_equal(o.read_qpel(), z["planes"])


def sad_case(encoder):
    z = npz("sad.npz")
    cur, ref = z["cur"], z["ref"]
    h, w = cur.shape
    cz = np.zeros((h // 2, w // 2), np.uint8)
    enc = encoder(w, h, int(z["sr"]))
    enc.set_reference(ref, cz, cz)
    return enc, (cur, cz, cz), z


def test_oracle_sad_table_matches_golden():
    o, cur, z = sad_case(lambda w, h, sr: oracle_lib.OracleEncoder(w, h, search_range=sr))
    o.load_current(*cur)
    assert np.array_equal(o.sad_table(z["mb_xy"], z["centres"]), z["table"])


# ---------------- MI355X path (GPU) ----------------
@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(MANIFEST["lencod"])))
def test_gpu_lencod_matches_golden(case):
    g = MANIFEST["lencod"][case]
    assert lencod_digests(LENCOD, g["params"]) == (g["bitstream_sha256"], g["recon_sha256"])


@pytest.mark.gpu
def test_gpu_sequence_matches_golden():
    assert sequence(lambda w, h, sr: jmhip.Encoder(w, h, search_range=sr)) == MANIFEST["sequence"]["pictures"]


@pytest.mark.gpu
def test_gpu_tq4x4_matches_golden():
    z = npz("tq4x4.npz")
    g = jmhip.Encoder(32, 32, search_range=4)
    for qp in (0, 12, 28, 51):
        for intra in (0, 1):
            got = g.tq4x4(z["resid"], z["pred"], qp, intra)
            for name, arr in zip(("lev", "rec", "cc", "nz"), got):
                assert np.array_equal(arr, z[f"{name}_{qp}_{intra}"]), (name, qp, intra)


@pytest.mark.gpu
def test_gpu_qpel_matches_golden():
    z = npz("qpel.npz")
    h, w = z["y"].shape
    g = jmhip.Encoder(w, h, search_range=4)
    g.set_reference(z["y"], z["u"], z["v"])
    assert np.array_equal(g.read_qpel(), z["planes"])


@pytest.mark.gpu
def test_gpu_sad_table_matches_golden():
    g, cur, z = sad_case(lambda w, h, sr: jmhip.Encoder(w, h, search_range=sr))
    g.load_frame(0, *cur)
    assert np.array_equal(g.sad_table(z["mb_xy"], z["centres"]), z["table"])

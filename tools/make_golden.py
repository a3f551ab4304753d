#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the oracle (CPU, no GPU).

  python tools/make_golden.py          # rewrite tests/golden/*

Fixtures (all data; no reference source text):
  manifest.json   sha256 of lencod_cpu bitstreams + reconstructions for eleven encoder.cfg
                  configurations (the first three as in the GPU bitstream test; one with slices, one
                  CABAC, two with RDOptimization 1 -- one of them High 10 -- and a High 10 RDO-off
                  one; round 4: RDO with CAVLC + FFS, RDO with the 8x8 transform at 10 bits, 10-bit
                  FFS), and of the
                  per-picture jmh_mb_result arrays + reconstructions of a 64x48 I-P-P sequence
  tq4x4.npz       dct_luma vectors: residual/prediction inputs and levels/recon/cost/nonzero
                  outputs at QP 0, 12, 28, 51, intra and inter rounding
  qpel.npz        a 48x32 reference picture and its 16 quarter-pel phase planes (8.4.2.2.1)
  sad.npz         SetupFastFullPelSearch 4x4 SAD tables (SR 8) for three MBs / window centres

The oracle's JM parity is unpinned (the reference repository holds no JM source, tests or
vectors): these fixtures pin the restatement against drift and let the GPU path be
checked against stored outputs without running the oracle.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402
from jmpaths import LENCOD_CPU, ensure_built, load_jmhip  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
LENCOD_CONFIGS = [
    ["InputFile=synthetic:1", "FramesToBeEncoded=10", "SourceWidth=176", "SourceHeight=144", "SearchRange=16"],
    ["InputFile=synthetic:2", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "IntraPeriod=3", "QPRemainingFrame=33"],
    ["InputFile=synthetic:3", "FramesToBeEncoded=3", "SourceWidth=200", "SourceHeight=120", "SearchRange=8",
     "LoopFilterParametersFlag=1", "LoopFilterAlphaC0Offset=2", "LoopFilterBetaOffset=-1"],
    # SliceMode 1 (docs/JM_SEMANTICS.md item 47): 22-MB slices, EPZS + 8x8 transform
    ["InputFile=synthetic:4", "FramesToBeEncoded=4", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=100", "Transform8x8Mode=1", "SearchMode=3", "SliceMode=1", "SliceArgument=22"],
    # CABAC (SymbolMode 1, docs/JM_SEMANTICS.md item 48): High, 8x8 transform, slices, an I picture every 3
    ["InputFile=synthetic:5", "FramesToBeEncoded=5", "SourceWidth=352", "SourceHeight=288", "SearchRange=32",
     "ProfileIDC=100", "Transform8x8Mode=1", "SymbolMode=1", "SliceMode=1", "SliceArgument=33", "IntraPeriod=3"],
    # RDOptimization 1 (items 53-60): CABAC RD loop, Main, EPZS, 11-MB slices
    ["InputFile=synthetic:6", "FramesToBeEncoded=4", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "ProfileIDC=77", "SymbolMode=1", "RDOptimization=1", "SearchMode=3", "SliceMode=1", "SliceArgument=11"],
    # config 5's shape: High 10 (ProfileIDC 110, 10-bit samples), CABAC RD loop, one-MB-row slices
    ["InputFile=synthetic:7", "FramesToBeEncoded=3", "SourceWidth=352", "SourceHeight=96", "SearchRange=32",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "SymbolMode=1", "RDOptimization=1",
     "SearchMode=3", "SliceMode=1", "SliceArgument=22", "QPRemainingFrame=30"],
    # High 10 with RDO off: EPZS + 8x8 transform, CAVLC
    ["InputFile=synthetic:8", "FramesToBeEncoded=3", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SearchMode=3"],
    # round 4: JM's default encoder.cfg shape -- RDOptimization 1 with CAVLC rates and FFS (items 64, 65)
    ["InputFile=synthetic:9", "FramesToBeEncoded=4", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "ProfileIDC=66", "RDOptimization=1", "SymbolMode=0", "SearchMode=0"],
    # RDOptimization 1 with the 8x8 transform at 10 bits (item 63): I8MB, 8x8-transform inter candidates
    ["InputFile=synthetic:10", "FramesToBeEncoded=3", "SourceWidth=352", "SourceHeight=96", "SearchRange=32",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SymbolMode=1",
     "RDOptimization=1", "SearchMode=3", "SliceMode=1", "SliceArgument=22"],
    # FFS on 10-bit samples, RDO off (item 66)
    ["InputFile=synthetic:11", "FramesToBeEncoded=3", "SourceWidth=176", "SourceHeight=144", "SearchRange=16",
     "ProfileIDC=110", "SourceBitDepthLuma=10", "SourceBitDepthChroma=10", "SearchMode=0"],
]
SEQ = dict(w=64, h=48, seed=21, frames=3, qp=28, search_range=16)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def run_lencod(binary, extra, out_dir):
    args = [binary, "-p", f"OutputFile={out_dir}/a.264", "-p", f"ReconFile={out_dir}/rec.yuv"]
    for e in extra:
        args += ["-p", e]
    subprocess.run(args, check=True, capture_output=True, timeout=600)
    return open(f"{out_dir}/a.264", "rb").read(), open(f"{out_dir}/rec.yuv", "rb").read()


def sequence_digests(encode):
    """encode(y, u, v, slice_type, qp) -> (results, recon); I then P pictures of SEQ."""
    jm = load_jmhip()
    out = []
    for i in range(SEQ["frames"]):
        pic = jm.synth_frame(SEQ["w"], SEQ["h"], SEQ["seed"], i)
        res, rec = encode(*pic, jm.JMH_I_SLICE if i == 0 else jm.JMH_P_SLICE, SEQ["qp"])
        out.append({"results": sha(res.tobytes()), "recon": sha(b"".join(p.tobytes() for p in rec))})
    return out


def oracle_sequence():
    o = oracle_lib.OracleEncoder(SEQ["w"], SEQ["h"], search_range=SEQ["search_range"])

    def enc(y, u, v, st, qp):
        res, rec = o.encode(y, u, v, st, qp)
        o.set_reference(*rec)
        return res, rec
    return sequence_digests(enc)


def main():
    ensure_built()
    os.makedirs(GOLD, exist_ok=True)
    rng = np.random.default_rng(20261015)
    manifest = {"provenance": "self-generated regression pins: outputs of this repository's oracle (lencod_cpu / "
                              "liboracle), not of JM; JM parity is unpinned (no JM source, binary or vectors "
                              "exist in the reference, DESIGN.md section 6)",
                "lencod": [], "sequence": {"spec": SEQ}}
    for extra in LENCOD_CONFIGS:
        with tempfile.TemporaryDirectory() as d:
            bs, rec = run_lencod(LENCOD_CPU, extra, d)
        manifest["lencod"].append({"kind": "regression_pin", "params": extra, "bitstream_sha256": sha(bs),
                                   "bitstream_bytes": len(bs),
                                   "recon_sha256": sha(rec), "bitstream_head_hex": bs[:48].hex()})
    manifest["sequence"]["pictures"] = oracle_sequence()
    with open(os.path.join(GOLD, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)

    n = 256
    resid = rng.integers(-255, 256, (n, 16)).astype(np.int16)
    resid[:8] = 255
    resid[8:16] = -255
    resid[16:24] = 0
    pred = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    arrays = {"resid": resid, "pred": pred}
    for qp in (0, 12, 28, 51):
        for intra in (0, 1):
            lev, rec, cc, nz = oracle_lib.tq4x4(resid, pred, qp, intra)
            arrays.update({f"lev_{qp}_{intra}": lev, f"rec_{qp}_{intra}": rec, f"cc_{qp}_{intra}": cc, f"nz_{qp}_{intra}": nz})
    np.savez_compressed(os.path.join(GOLD, "tq4x4.npz"), **arrays)

    w, h = 48, 32
    ref = [rng.integers(0, 256, (h, w)).astype(np.uint8), rng.integers(0, 256, (h // 2, w // 2)).astype(np.uint8),
           rng.integers(0, 256, (h // 2, w // 2)).astype(np.uint8)]
    o = oracle_lib.OracleEncoder(w, h, search_range=4)
    o.set_reference(*ref)
    np.savez_compressed(os.path.join(GOLD, "qpel.npz"), y=ref[0], u=ref[1], v=ref[2], planes=o.read_qpel())

    w, h, sr = 64, 48, 8
    cur = [rng.integers(0, 256, (h, w)).astype(np.uint8), np.zeros((h // 2, w // 2), np.uint8), np.zeros((h // 2, w // 2), np.uint8)]
    ref = [np.clip(cur[0].astype(int) + rng.integers(-9, 10, (h, w)), 0, 255).astype(np.uint8), cur[1], cur[2]]
    o = oracle_lib.OracleEncoder(w, h, search_range=sr)
    o.set_reference(*ref)
    o.load_current(*cur)
    mb_xy = np.array([(0, 0), (3, 2), (1, 1)], np.int32)
    centres = np.array([(0, 0), (-sr, sr), (3, -2)], np.int32)
    np.savez_compressed(os.path.join(GOLD, "sad.npz"), cur=cur[0], ref=ref[0], mb_xy=mb_xy, centres=centres, sr=np.int32(sr),
                        table=o.sad_table(mb_xy, centres))
    print("wrote", sorted(os.listdir(GOLD)))


if __name__ == "__main__":
    main()

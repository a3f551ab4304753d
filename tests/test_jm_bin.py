"""The JM parity hook (SURVEY.md §4 "JM parity"): with `--jm-bin PATH` (and optionally
`--jm-cfg` for that build's own encoder.cfg and `--jm-version`), every case below encodes the same
synthetic I420 file with the JM lencod and with this build's CPU lencod (lencod_cpu; the GPU
lencod is pinned byte-equal to it by tests/test_gpu_parity.py) and requires the two .264 files and
the two reconstructions to be byte-identical.

No JM binary or source exists in this pipeline, so without `--jm-bin` every case is skipped: the
hook is wired, not exercised.  Case keys use the JM 8.6 spellings both builds read; keys only JM
needs (FrameSkip, NumberBFrames, ...) go to JM alone, and this build's JMVersion knob is set from
`--jm-version`."""
import os
import subprocess
import tempfile

import pytest

from jmpaths import LENCOD_CPU, ensure_built, load_jmhip

jmhip = load_jmhip()

# (this build's keys, JM-only keys, minimum JM major version)
CASES = [
    # config 1 shape: QCIF IPPP, fast full search SR 16, Baseline
    (["SourceWidth=176", "SourceHeight=144", "FramesToBeEncoded=10", "SearchRange=16", "QPFirstFrame=28",
      "QPRemainingFrame=28"], ["FrameSkip=0", "NumberBFrames=0", "RDOptimization=0", "SymbolMode=0"], 8),
    (["SourceWidth=176", "SourceHeight=144", "FramesToBeEncoded=5", "SearchRange=8", "UseHadamard=0",
      "IntraPeriod=3", "QPFirstFrame=24", "QPRemainingFrame=30"],
     ["FrameSkip=0", "NumberBFrames=0", "RDOptimization=0", "SymbolMode=0"], 8),
    (["SourceWidth=352", "SourceHeight=288", "FramesToBeEncoded=4", "SearchRange=32", "LoopFilterParametersFlag=1",
      "LoopFilterAlphaC0Offset=2", "LoopFilterBetaOffset=-1"],
     ["FrameSkip=0", "NumberBFrames=0", "RDOptimization=0", "SymbolMode=0"], 8),
    # config 3 shape (JM >= 10): High profile, 8x8 transform, EPZS
    (["SourceWidth=352", "SourceHeight=288", "FramesToBeEncoded=4", "SearchRange=32", "ProfileIDC=100",
      "Transform8x8Mode=1", "SearchMode=3"],
     ["FrameSkip=0", "NumberBFrames=0", "RDOptimization=0", "SymbolMode=0", "AdaptiveRounding=0",
      "OffsetMatrixPresentFlag=0", "EPZSPattern=2", "EPZSDualRefinement=0", "EPZSFixedPredictors=2",
      "EPZSTemporal=1", "EPZSSpatialMem=1", "EPZSSubPelME=0"], 10),
]


@pytest.fixture
def jm(request):
    path = request.config.getoption("--jm-bin")
    if not path:
        pytest.skip("no --jm-bin given (no JM build exists in this pipeline)")
    assert os.access(path, os.X_OK), f"--jm-bin {path} is not executable"
    return path, request.config.getoption("--jm-cfg"), request.config.getoption("--jm-version")


def write_yuv(path, w, h, n, seed):
    with open(path, "wb") as f:
        for i in range(n):
            y, u, v = jmhip.synth_frame(w, h, seed, i)
            f.write(y[:h, :w].tobytes() + u[:h // 2, :w // 2].tobytes() + v[:h // 2, :w // 2].tobytes())


def key(params, k):
    return int(next(p.split("=", 1)[1] for p in params if p.startswith(k + "=")))


def run_case(jm_bin, jm_cfg, jm_version, ours, jm_only):
    ensure_built()
    w, h, n = key(ours, "SourceWidth"), key(ours, "SourceHeight"), key(ours, "FramesToBeEncoded")
    with tempfile.TemporaryDirectory() as d:
        write_yuv(f"{d}/in.yuv", w, h, n, seed=11)
        io = lambda tag: [f"InputFile={d}/in.yuv", f"OutputFile={d}/{tag}.264", f"ReconFile={d}/{tag}_rec.yuv"]
        args = [jm_bin] + (["-d", jm_cfg] if jm_cfg else [])
        for p in io("jm") + ours + jm_only:
            args += ["-p", p]
        r = subprocess.run(args, capture_output=True, text=True, timeout=3600, cwd=d)   # JM writes its stats into cwd
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        args = [LENCOD_CPU]
        for p in io("ours") + ours + [f"JMVersion={jm_version}"]:
            args += ["-p", p]
        r = subprocess.run(args, capture_output=True, text=True, timeout=3600)
        assert r.returncode == 0, r.stdout + r.stderr
        assert open(f"{d}/ours.264", "rb").read() == open(f"{d}/jm.264", "rb").read(), "bitstreams differ from JM"
        assert open(f"{d}/ours_rec.yuv", "rb").read() == open(f"{d}/jm_rec.yuv", "rb").read(), "recon differs from JM"


@pytest.mark.parametrize("ours,jm_only,min_version", CASES, ids=[f"case{i}" for i in range(len(CASES))])
def test_bitstream_and_recon_equal_jm(jm, ours, jm_only, min_version):
    jm_bin, jm_cfg, jm_version = jm
    if jm_version < min_version:
        pytest.skip(f"needs a JM >= {min_version} build")
    run_case(jm_bin, jm_cfg, jm_version, ours, jm_only)


STAND_IN = """#!/bin/sh
# stand-in for a JM lencod (hook plumbing test only): drops the JM-only keys, runs lencod_cpu
skip="FrameSkip NumberBFrames RDOptimization SymbolMode AdaptiveRounding OffsetMatrixPresentFlag EPZSPattern
EPZSDualRefinement EPZSFixedPredictors EPZSTemporal EPZSSpatialMem EPZSSubPelME"
set -- "$@"
out=""
while [ $# -gt 0 ]; do
  if [ "$1" = "-p" ]; then
    k=${2%%=*}; keep=1
    for s in $skip; do [ "$k" = "$s" ] && keep=0; done
    [ $keep = 1 ] && out="$out -p $2"
    shift 2
  else
    out="$out $1"; shift
  fi
done
exec %s $out -p JMVersion=%d
"""


@pytest.mark.parametrize("version,case", [(8, 0), (10, 3)])
def test_hook_plumbing_with_a_stand_in_binary(version, case):
    """The hook itself runs: a stand-in 'JM' (this build's lencod_cpu behind a key filter) must
    compare equal through run_case for a JM 8.6 and a JM >= 10 case."""
    ensure_built()
    with tempfile.TemporaryDirectory() as d:
        path = f"{d}/lencod_stand_in"
        with open(path, "w") as f:
            f.write(STAND_IN % (LENCOD_CPU, version))
        os.chmod(path, 0o755)
        ours, jm_only, _ = CASES[case]
        run_case(path, None, version, ["FramesToBeEncoded=2" if p.startswith("FramesToBeEncoded") else p for p in ours],
                 jm_only)

"""The product's CABAC and CAVLC rate engines against independent counts, candidate by candidate
(row f4, parity of the RD decision).

csrc/jmh_cabac_rate.h is the text the RD kernels (k_rdo_inter / k_rdo_intra / k_rdo_final) compile:
it counts renormalisation steps over a dense context space.  The oracle prices RD candidates with its
own CABAC coder (oracle/cabac_enc.c: 9.3.4.2 with codILow, PutBit / outstanding bits, JM's
arienco_bits_written, the decoder's context tables, spec ctxIdx numbering) and shares no code with
it.  tests/harness/lencod_xcheck runs the CPU lencod with a hook on every rate the oracle's RD loop
computes -- P_Skip and macroblock candidates, every 8x8 sub-mode, every Intra4x4 mode, the losing
ones included -- and requires the product engine's bit count, context states and codIRange from the
same stored state to be identical.  The writer check of test_rdo.py covers only each macroblock's
chosen candidate; this covers the candidates that lose, whose wrong rate would flip decisions on
the device and in the oracle alike.
"""
import re
import subprocess
import tempfile

import pytest

from jmpaths import LENCOD_XCHECK, ensure_built
from test_rdo import BASE, CAVLC, RDO

XCHECK = RDO + [
    # config 5's slice structure at its real width: 240-MB (one row) slices, High 10 and 8-bit
    ["InputFile=synthetic:83", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=10",
     "SourceBitDepthChroma=10", "SourceWidth=3840", "SourceHeight=48", "SearchRange=32", "SliceMode=1",
     "SliceArgument=240"],
    ["InputFile=synthetic:84", "FramesToBeEncoded=3", "ProfileIDC=77", "SourceWidth=3840", "SourceHeight=48",
     "SearchRange=32", "SliceMode=1", "SliceArgument=240", "QPRemainingFrame=22"],
    # JM >= 10 EPZS options under RDO, low QP (long level codes: the UEG0 suffix of the rate)
    ["InputFile=synthetic:85", "FramesToBeEncoded=3", "ProfileIDC=77", "SearchRange=16", "EPZSSubPelME=1",
     "EPZSMaxThresScale=2", "QPFirstFrame=4", "QPRemainingFrame=6"],
    # Transform8x8Mode 1 with RDO (item 63): I8MB by RDCost_for_8x8IntraBlocks, 8x8-transform inter candidates
    ["InputFile=synthetic:86", "FramesToBeEncoded=4", "ProfileIDC=100", "Transform8x8Mode=1", "SearchRange=16"],
    ["InputFile=synthetic:87", "FramesToBeEncoded=3", "ProfileIDC=100", "Transform8x8Mode=1", "SearchRange=8",
     "QPFirstFrame=8", "QPRemainingFrame=10", "SliceMode=1", "SliceArgument=5"],
    ["InputFile=synthetic:88", "FramesToBeEncoded=3", "ProfileIDC=110", "SourceBitDepthLuma=10",
     "SourceBitDepthChroma=10", "Transform8x8Mode=1", "SourceWidth=3840", "SourceHeight=48", "SearchRange=32",
     "SliceMode=1", "SliceArgument=240"],
]


def run_xcheck(extra, base=BASE):
    with tempfile.TemporaryDirectory() as d:
        args = [LENCOD_XCHECK, "-p", f"OutputFile={d}/a.264"]
        for e in base + extra:
            args += ["-p", e]
        r = subprocess.run(args, capture_output=True, text=True, timeout=900)
    log = r.stdout + r.stderr
    m = re.search(r"rate xcheck: (\d+) candidates \(skip (\d+), mb (\d+), b8 (\d+), i4 (\d+), i8 (\d+)\), (\d+) mismatches",
                  log)
    assert m, log[-3000:]
    return r.returncode, [int(v) for v in m.groups()], log


@pytest.mark.parametrize("extra", XCHECK, ids=[c[0].split(":")[1] for c in XCHECK])
def test_rate_engine_equals_oracle_coder_on_every_candidate(extra):
    ensure_built()
    rc, (n, skip, mb, b8, i4, i8, bad), log = run_xcheck(extra)
    assert rc == 0 and bad == 0, log[-3000:]
    assert n > 0 and mb > 0 and i4 > 0, log[-3000:]
    if "IntraPeriod=1" not in extra:                       # P pictures: skip and P8x8 candidates too
        assert skip > 0 and b8 > 0, log[-3000:]
    if "Transform8x8Mode=1" in extra:                      # Intra8x8 candidates
        assert i8 > 0, log[-3000:]


@pytest.mark.parametrize("extra", CAVLC, ids=[c[0].split(":")[1] for c in CAVLC])
def test_cavlc_rate_engine_equals_oracle_count_on_every_candidate(extra):
    """SymbolMode 0 (item 64): csrc/jmh_cavlc_rate.h against oracle/cavlc_bits.c, every candidate."""
    ensure_built()
    rc, (n, skip, mb, b8, i4, i8, bad), log = run_xcheck(extra, ["SymbolMode=0", "RDOptimization=1", "SearchMode=3"])
    assert rc == 0 and bad == 0, log[-3000:]
    assert n > 0 and mb > 0 and i4 > 0, log[-3000:]

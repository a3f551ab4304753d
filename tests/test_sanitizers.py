"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the host code: the CPU
encoder (tests/harness/lencod_cpu.c driving the product's host plumbing — cfg, yuv, bitstream, deblock,
encoder loop with its writer threads, the JM 8.6 call surface) and the spec decoder, built by
`make -C tests/harness sanitize` with -fsanitize=address,undefined -fno-sanitize-recover=undefined, on
the closed-loop configurations.  Any report aborts the process, so a clean exit plus the
closed-loop equality (decoder output == encoder reconstruction) is the check.  GPU-side ASan is
not available on this pool; the device code is covered by the parity tests instead."""
import fcntl
import os
import subprocess
import tempfile

import pytest

from jmpaths import HARNESS
from test_closed_loop import CABAC, CONFIGS

ASAN = os.path.join(HARNESS, "_build_asan")
LENCOD_ASAN = os.path.join(ASAN, "lencod_cpu")
JMDEC_ASAN = os.path.join(ASAN, "jmdec")

# the sanitized binaries are ~5-10x slower: a subset of the closed-loop shapes plus the host
# surfaces the plain closed-loop test does not drive (writer threads, JM call surface)
SAN_CASES = [CONFIGS[0], CONFIGS[1], CONFIGS[4], CONFIGS[6], CONFIGS[7], CONFIGS[12], CONFIGS[15], CONFIGS[16],
             CONFIGS[0] + ["WriterThreads=4"],
             CONFIGS[6] + ["JMCallSurface=1"],
             CONFIGS[12] + ["WriterThreads=0", "JMCallSurface=1"],
             CONFIGS[19] + ["WriterThreads=4"],                # SliceMode 1 (several NAL units per picture)
             CONFIGS[20] + ["JMCallSurface=1"],
             CABAC[0], CABAC[2], CABAC[5], CABAC[7] + ["WriterThreads=4"]]   # CABAC coder + parser

ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")


@pytest.fixture(scope="module")
def sanitized():
    # one build at a time (pytest-xdist workers each run this fixture)
    with open(os.path.join(HARNESS, ".sanitize.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", HARNESS, "sanitize"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stdout + r.stderr)
    return LENCOD_ASAN, JMDEC_ASAN


@pytest.mark.parametrize("extra", SAN_CASES, ids=[f"{c[0].split(':')[1]}-{len(c)}" for c in SAN_CASES])
def test_sanitized_encode_decode(sanitized, extra):
    enc, dec = sanitized
    with tempfile.TemporaryDirectory() as d:
        args = [enc, "-p", f"OutputFile={d}/a.264", "-p", f"ReconFile={d}/rec.yuv"]
        for e in extra:
            args += ["-p", e]
        r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=ENV)
        log = r.stdout + r.stderr
        assert r.returncode == 0 and "runtime error" not in log and "Sanitizer" not in log, log[-4000:]
        r = subprocess.run([dec, f"{d}/a.264", f"{d}/dec.yuv"], capture_output=True, text=True, timeout=600, env=ENV)
        log = r.stdout + r.stderr
        assert r.returncode == 0 and "runtime error" not in log and "Sanitizer" not in log, log[-4000:]
        assert open(f"{d}/dec.yuv", "rb").read() == open(f"{d}/rec.yuv", "rb").read()

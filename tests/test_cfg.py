"""encoder.cfg interface (JM configfile.c semantics): Key = Value, comments, -f/-p order,
unknown keys and unsupported settings are errors."""
import subprocess
import tempfile

from jmpaths import LENCOD_CPU, ensure_built


def run(*args):
    ensure_built()
    return subprocess.run([LENCOD_CPU, *args], capture_output=True, text=True, timeout=120)


def test_cfg_file_and_override_order():
    with tempfile.TemporaryDirectory() as d:
        cfg = f"{d}/encoder.cfg"
        with open(cfg, "w") as f:
            f.write("# JM-style config\nInputFile = \"synthetic:4\"   # quoted\nFramesToBeEncoded = 2\n"
                    "SourceWidth = 64\nSourceHeight = 48\nSearchRange = 4\nQPFirstFrame = 30\n"
                    f"OutputFile = {d}/o.264\n")
        r = run("-d", cfg, "-p", "QPFirstFrame=31")
        assert r.returncode == 0, r.stderr
        assert " 31 " in r.stdout.splitlines()[2]          # override applied after the file


def test_unknown_key_is_error():
    r = run("-p", "NoSuchKey=1")
    assert r.returncode != 0 and "not recognized" in r.stderr


def test_range_checked():
    r = run("-p", "SearchRange=999")
    assert r.returncode != 0 and "out of range" in r.stderr


def test_unsupported_rdo_reported():
    r = run("-p", "RDOptimization=2")   # RDOptimization 1 runs with every entropy coder and search mode
    assert r.returncode != 0 and "RDOptimization" in r.stderr


def test_jm86_spellings_accepted():
    with tempfile.TemporaryDirectory() as d:
        r = run("-p", "UseFME=0", "-p", "QPRemainingFrame=30", "-p", "FramesToBeEncoded=1", "-p", "SourceWidth=32",
                "-p", "SourceHeight=32", "-p", "SearchRange=2", "-p", f"OutputFile={d}/o.264")
        assert r.returncode == 0, r.stderr


def test_transform8x8_requires_high_profile():
    r = run("-p", "Transform8x8Mode=1")
    assert r.returncode != 0 and "ProfileIDC=100" in r.stderr
    r = run("-p", "ProfileIDC=88")
    assert r.returncode != 0 and "ProfileIDC" in r.stderr
    r = run("-p", "ProfileIDC=77", "-p", "Transform8x8Mode=1")
    assert r.returncode != 0 and "ProfileIDC=100" in r.stderr


def test_cabac_keys():
    """SymbolMode 1 (CABAC) needs Main / High; the adaptive context initialisation and
    cabac_init_idc 1 / 2 are rejected loudly (docs/JM_SEMANTICS.md item 48)."""
    r = run("-p", "SymbolMode=1")
    assert r.returncode != 0 and "Baseline" in r.stderr
    r = run("-p", "SymbolMode=1", "-p", "ProfileIDC=77", "-p", "ContextInitMethod=1")
    assert r.returncode != 0 and "ContextInitMethod" in r.stderr
    r = run("-p", "SymbolMode=1", "-p", "ProfileIDC=77", "-p", "FixedModelNumber=2")
    assert r.returncode != 0 and "FixedModelNumber" in r.stderr
    with tempfile.TemporaryDirectory() as d:
        r = run("-p", "SymbolMode=1", "-p", "ProfileIDC=77", "-p", "FramesToBeEncoded=2", "-p", "SourceWidth=64",
                "-p", "SourceHeight=48", "-p", "SearchRange=2", "-p", f"OutputFile={d}/o.264")
        assert r.returncode == 0, r.stderr


def test_slice_mode_keys():
    """SliceMode 1 / SliceArgument accepted; byte-count slices (2) and slice groups (3) rejected,
    SliceArgument range-checked."""
    r = run("-p", "SliceMode=2")
    assert r.returncode != 0 and "SliceMode=2" in r.stderr
    r = run("-p", "SliceMode=1", "-p", "SliceArgument=0")
    assert r.returncode != 0 and "out of range" in r.stderr
    with tempfile.TemporaryDirectory() as d:
        r = run("-p", "SliceMode=1", "-p", "SliceArgument=3", "-p", "FramesToBeEncoded=1", "-p", "SourceWidth=64",
                "-p", "SourceHeight=48", "-p", "SearchRange=2", "-p", f"OutputFile={d}/o.264")
        assert r.returncode == 0, r.stderr

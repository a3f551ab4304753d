"""Locations of the built artefacts and loaders for tests (the package dir has a '-' in it)."""
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "h264-jm-commentary_amd")
ORACLE = os.path.join(ROOT, "oracle")
LIBJMHIP = os.path.join(PKG, "csrc", "libjmhip.so")
LIBJMHOST = os.path.join(PKG, "host", "build", "libjmhost.so")
LENCOD = os.path.join(PKG, "host", "build", "lencod")
LIBORACLE = os.path.join(ORACLE, "_build", "liboracle.so")
HARNESS = os.path.join(ROOT, "tests", "harness")
LENCOD_CPU = os.path.join(HARNESS, "_build", "lencod_cpu")
LENCOD_XCHECK = os.path.join(HARNESS, "_build", "lencod_xcheck")
JMDEC = os.path.join(ORACLE, "_build", "jmdec")
JM86_CHECK = os.path.join(HARNESS, "_build", "jm86_check")
HEADER = os.path.join(ROOT, "include", "jmhip.h")


def ensure_built():
    need = [LIBJMHOST, LIBORACLE, LENCOD_CPU, LENCOD_XCHECK, JMDEC]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-s", "-C", ROOT, "harness"], check=True)


def load_jmhip():
    if "jmhip" in sys.modules:
        return sys.modules["jmhip"]
    spec = importlib.util.spec_from_file_location("jmhip", os.path.join(PKG, "jmhip.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["jmhip"] = mod
    spec.loader.exec_module(mod)
    return mod

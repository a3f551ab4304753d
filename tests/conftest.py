import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running (full 1080p oracle frames)")


def pytest_addoption(parser):
    # SURVEY.md §4 "JM parity": run tests/test_jm_bin.py against a JM lencod the moment one exists
    parser.addoption("--jm-bin", default=None,
                     help="path to a JM lencod binary: enables tests/test_jm_bin.py (bitstream and recon "
                          "byte-equality with this build's lencod for the same encoder.cfg)")
    parser.addoption("--jm-cfg", default=None,
                     help="the JM build's own encoder.cfg, passed with -d before the -p overrides")
    parser.addoption("--jm-version", default=8, type=int,
                     help="major version of the --jm-bin build (8 = JM 8.6; >= 10 enables the FRExt / EPZS cases "
                          "and runs this build with JMVersion=<value>)")

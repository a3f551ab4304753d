import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running (full 1080p oracle frames)")

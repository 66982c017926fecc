"""Test configuration.

Markers:
  gpu  — needs an MI355X (run with `pytest -m gpu`); everything else runs on CPU.
Paths: the product binding (peter-shirley-ray-tracing-the-next-week_amd/rtnw.py) and
the test-only oracle (oracle/oracle.py).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950)")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)

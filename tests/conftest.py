"""pytest configuration: the ``gpu`` marker and import paths.

``-m "not gpu"``: oracle vs golden vectors, host logic, C-ABI library loads and
exports every declared symbol, multi-process (gloo) host paths.
``-m gpu``: parity of the HIP path (through the C ABI) against the oracle.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cugraph-forked_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "reference_vectors.json")) as f:
        return json.load(f)


def dataset_path(name):
    return os.path.join(GOLDEN, name)

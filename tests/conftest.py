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


_T0 = None


def pytest_runtest_logstart(nodeid, location):
    """CGX_TEST_CLOCK=1: print the suite's elapsed seconds as each test starts (a
    killed or hung GPU run's log then says when it stopped)."""
    global _T0
    if os.environ.get("CGX_TEST_CLOCK") != "1":
        return
    import time
    now = time.monotonic()
    if _T0 is None:
        _T0 = now
    sys.stdout.write(f"\n[{now - _T0:7.1f} s] ")
    sys.stdout.flush()


def pytest_collection_modifyitems(session, config, items):
    """The multi-rank rehearsals (tests/test_gpu_mg.py, every GPU call in spawned
    ranks) run before any test that opens a HIP context in the pytest process itself.
    Measured on the one-GPU box: a world-8 rehearsal takes 4-5 s when pytest has no
    context of its own, and 73-153 s after in-process GPU tests (bench-parity module
    first, caches trimmed, GPU_MAX_HW_QUEUES=2 in the ranks made no difference) -- all
    8 ranks then spin at 100 % CPU on their staged copies."""
    first = [i for i in items if i.fspath.basename == "test_gpu_mg.py"]
    if first:
        rest = [i for i in items if i.fspath.basename != "test_gpu_mg.py"]
        items[:] = first + rest

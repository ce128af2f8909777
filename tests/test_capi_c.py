"""The plain-C boundary client (tests/c/capi_test.c): compiled with gcc against
include/cugraph_c/*.h and linked to libcugraph_c.so -- the way a C caller of the
reference's libcugraph_c would build -- and run on the GPU.  It re-authors the
reference's cpp/tests/c_api/{pagerank,bfs,sssp,louvain}_test.c cases."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG, ROOT

SRC = os.path.join(ROOT, "tests", "c", "capi_test.c")
BIN = os.path.join(ROOT, "tests", "c", "capi_test")
LIBDIR = os.path.join(PKG, "lib")


@pytest.mark.skipif(not os.path.exists(os.path.join(LIBDIR, "libcugraph_c.so")) or not shutil.which("gcc"),
                    reason="library not built / no gcc")
def test_c_client_compiles_and_links(tmp_path):
    out = tmp_path / "capi_test"
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                        "-o", str(out), SRC, "-L", LIBDIR, "-lcugraph_c", "-lm", f"-Wl,-rpath,{LIBDIR}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_c_client_runs():
    assert os.path.exists(BIN), "tests/c/capi_test not built (make -C cugraph-forked_amd)"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("pagerank", "personalized_pagerank", "bfs", "sssp", "louvain", "errors", "release"):
        assert f"PASS {name}" in r.stdout

"""CPU-side checks of the drop-in boundary: the built libcugraph_c.so loads and
exports every function declared in include/cugraph_c/*.h and include/cugraph_amd/*.h
(no GPU calls)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT

LIB = os.path.join(PKG, "lib", "libcugraph_c.so")


def declared_functions():
    names = set()
    for sub in ("cugraph_c", "cugraph_amd"):
        d = os.path.join(ROOT, "include", sub)
        for f in sorted(os.listdir(d)):
            if not f.endswith(".h"):
                continue
            text = open(os.path.join(d, f)).read()
            text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
            for m in re.finditer(r"\b(cugraph_\w+)\s*\(", text):
                names.add(m.group(1))
    return sorted(names)


def test_headers_declare_reference_entry_points():
    names = set(declared_functions())
    for must in ["cugraph_create_resource_handle", "cugraph_sg_graph_create", "cugraph_mg_graph_create",
                 "cugraph_pagerank", "cugraph_personalized_pagerank", "cugraph_bfs", "cugraph_sssp",
                 "cugraph_louvain", "cugraph_centrality_result_get_values", "cugraph_paths_result_get_distances",
                 "cugraph_heirarchical_clustering_result_get_modularity", "cugraph_error_message",
                 "cugraph_type_erased_device_array_view_copy_to_host",
                 "cugraph_type_erased_device_array_release", "cugraph_type_erased_host_array_release"]:
        assert must in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert missing == []


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built")
def test_python_shim_imports_without_gpu():
    import pylibcugraph
    assert "gfx950" in pylibcugraph.version()
    # mirrors the reference's pylibcugraph entry points
    for n in ["ResourceHandle", "GraphProperties", "SGGraph", "MGGraph", "pagerank",
              "personalized_pagerank", "bfs", "sssp", "louvain"]:
        assert hasattr(pylibcugraph, n)

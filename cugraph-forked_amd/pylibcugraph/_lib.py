"""ctypes binding of libcugraph_c (the MI355X build in ../lib/libcugraph_c.so).

Plays the role of the reference's Cython declarations
(``python/pylibcugraph/pylibcugraph/_cugraph_c/*.pxd``) and ``utils.pyx``
(``assert_success`` at ``utils.pyx:37-80``, ``copy_to_cupy_array`` at
``utils.pyx:150-184``).  There is no fallback: if the HIP library is missing the
import fails loudly.
"""
from __future__ import annotations

import atexit
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "CUGRAPH_AMD_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libcugraph_c.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libcugraph_c.so not found at {LIB_PATH}: build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C cugraph-forked_amd`)")

# torch bundles its own HIP runtime (torch/lib/libamdhip64.so, loaded by path).  Load
# it FIRST so that libcugraph_c's DT_NEEDED libamdhip64.so.7 / libhsa-runtime64.so.1
# resolve to the same, already-loaded objects: one HIP runtime per process.  (Loading
# ours first makes torch load a second runtime: two HIP runtimes in one process
# corrupt the heap at exit.)
try:
    import torch  # noqa: F401
except ImportError:  # pure C-ABI use without torch: the system ROCm runtime is used
    torch = None

lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)

# Objects still alive at interpreter exit are not freed (the process is going
# away; calling into HIP during teardown is not safe).
SHUTDOWN = [False]
atexit.register(lambda: SHUTDOWN.__setitem__(0, True))

# enums (include/cugraph_c/resource_handle.h, error.h)
INT32, INT64, FLOAT32, FLOAT64 = 0, 1, 2, 3
CODES = {
    0: "CUGRAPH_SUCCESS", 1: "CUGRAPH_UNKNOWN_ERROR", 2: "CUGRAPH_INVALID_HANDLE",
    3: "CUGRAPH_ALLOC_ERROR", 4: "CUGRAPH_INVALID_INPUT", 5: "CUGRAPH_NOT_IMPLEMENTED",
    6: "CUGRAPH_UNSUPPORTED_TYPE_COMBINATION",
}

P = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
c_size_t = ctypes.c_size_t
c_int = ctypes.c_int
c_double = ctypes.c_double


class GraphPropertiesStruct(ctypes.Structure):
    _fields_ = [("is_symmetric", ctypes.c_int), ("is_multigraph", ctypes.c_int)]


def _proto(name, restype, *argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)
    return f


# resource handle / errors
_proto("cugraph_create_resource_handle", P, P)
_proto("cugraph_free_resource_handle", None, P)
_proto("cugraph_resource_handle_get_rank", c_int, P)
_proto("cugraph_error_message", ctypes.c_char_p, P)
_proto("cugraph_error_free", None, P)
# arrays
_proto("cugraph_type_erased_device_array_create", c_int, P, c_size_t, c_int, PP, PP)
_proto("cugraph_type_erased_device_array_free", None, P)
_proto("cugraph_type_erased_device_array_view", P, P)
_proto("cugraph_type_erased_device_array_view_create", P, P, c_size_t, c_int)
_proto("cugraph_type_erased_device_array_view_free", None, P)
_proto("cugraph_type_erased_device_array_view_size", c_size_t, P)
_proto("cugraph_type_erased_device_array_view_type", c_int, P)
_proto("cugraph_type_erased_device_array_view_pointer", P, P)
_proto("cugraph_type_erased_device_array_view_copy", c_int, P, P, P, PP)
_proto("cugraph_type_erased_device_array_view_copy_to_host", c_int, P, P, P, PP)
_proto("cugraph_type_erased_device_array_view_copy_from_host", c_int, P, P, P, PP)
# graphs
_proto("cugraph_sg_graph_create", c_int, P, ctypes.POINTER(GraphPropertiesStruct), P, P, P, P, P,
       c_int, c_int, c_int, PP, PP)
_proto("cugraph_sg_graph_free", None, P)
_proto("cugraph_mg_graph_create", c_int, P, ctypes.POINTER(GraphPropertiesStruct), P, P, P, P, P,
       c_int, c_size_t, c_int, PP, PP)
_proto("cugraph_mg_graph_free", None, P)
# algorithms
_proto("cugraph_pagerank", c_int, P, P, P, P, P, P, c_double, c_double, c_size_t, c_int, PP, PP)
_proto("cugraph_personalized_pagerank", c_int, P, P, P, P, P, P, P, P, c_double, c_double, c_size_t,
       c_int, PP, PP)
_proto("cugraph_centrality_result_get_vertices", P, P)
_proto("cugraph_centrality_result_get_values", P, P)
_proto("cugraph_centrality_result_free", None, P)
_proto("cugraph_katz_centrality", c_int, P, P, P, c_double, c_double, c_double, c_size_t, c_int, PP, PP)
_proto("cugraph_eigenvector_centrality", c_int, P, P, c_double, c_size_t, c_int, PP, PP)
_proto("cugraph_hits", c_int, P, P, c_double, c_size_t, P, P, c_int, c_int, PP, PP)
_proto("cugraph_hits_result_get_vertices", P, P)
_proto("cugraph_hits_result_get_hubs", P, P)
_proto("cugraph_hits_result_get_authorities", P, P)
_proto("cugraph_hits_result_get_hub_score_differences", c_double, P)
_proto("cugraph_hits_result_get_number_of_iterations", c_size_t, P)
_proto("cugraph_hits_result_free", None, P)
_proto("cugraph_extract_paths", c_int, P, P, P, P, P, PP, PP)
_proto("cugraph_extract_paths_result_get_max_path_length", c_size_t, P)
_proto("cugraph_extract_paths_result_get_paths", P, P)
_proto("cugraph_extract_paths_result_free", None, P)
_proto("cugraph_bfs", c_int, P, P, P, c_int, c_size_t, c_int, c_int, PP, PP)
_proto("cugraph_sssp", c_int, P, P, c_size_t, c_double, c_int, c_int, PP, PP)
_proto("cugraph_paths_result_get_vertices", P, P)
_proto("cugraph_paths_result_get_distances", P, P)
_proto("cugraph_paths_result_get_predecessors", P, P)
_proto("cugraph_paths_result_free", None, P)
_proto("cugraph_louvain", c_int, P, P, c_size_t, c_double, c_int, PP, PP)
_proto("cugraph_heirarchical_clustering_result_get_vertices", P, P)
_proto("cugraph_heirarchical_clustering_result_get_clusters", P, P)
_proto("cugraph_heirarchical_clustering_result_get_modularity", c_double, P)
_proto("cugraph_heirarchical_clustering_result_free", None, P)
_proto("cugraph_amd_heirarchical_clustering_result_get_num_levels", c_size_t, P)
_proto("cugraph_amd_heirarchical_clustering_result_get_level", P, P, c_size_t)
# extensions (include/cugraph_amd/ext.h)
_proto("cugraph_amd_generate_rmat_edgelist", c_int, P, c_size_t, c_size_t, c_double, c_double, c_double,
       ctypes.c_uint64, c_int, c_int, c_size_t, c_int, PP, PP, PP)
_proto("cugraph_amd_generate_edge_weights", c_int, P, c_size_t, ctypes.c_uint64, c_size_t, c_int, PP, PP)
_proto("cugraph_amd_symmetrize_dedup", c_int, P, P, P, P, c_int, PP, PP, PP, PP)
_proto("cugraph_amd_graph_get_number_of_vertices", ctypes.c_int64, P)
_proto("cugraph_amd_graph_get_number_of_edges", ctypes.c_int64, P)
_proto("cugraph_amd_graph_is_symmetric", c_int, P)
_proto("cugraph_amd_graph_get_adjacency", c_int, P, P, c_int, PP, PP, PP, PP)
_proto("cugraph_amd_graph_get_out_weight_sums", c_int, P, P, PP, PP)
_proto("cugraph_amd_device_array_views_copy", c_int, P, c_size_t, P, P, PP)
_proto("cugraph_amd_set_profiling", None, P, c_int)
_proto("cugraph_amd_set_option", c_int, P, ctypes.c_char_p, c_double, PP)
_proto("cugraph_amd_last_iterations", c_size_t, P)
_proto("cugraph_amd_last_hot_kernel_ms", c_double, P)
_proto("cugraph_amd_last_hot_kernel_launches", c_size_t, P)
_proto("cugraph_amd_last_bfs_levels", c_size_t, P)
_proto("cugraph_amd_last_bfs_bottom_up_steps", c_size_t, P)
_proto("cugraph_amd_last_louvain_levels", c_size_t, P)
_proto("cugraph_amd_last_louvain_sweep_bytes", c_double, P)
_proto("cugraph_amd_last_louvain_partition", None, P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64))
_proto("cugraph_amd_trim_device_cache", c_size_t)
_proto("cugraph_amd_allocator_stats", None, ctypes.POINTER(c_double))
_proto("cugraph_amd_version", ctypes.c_char_p)
_proto("cugraph_amd_measure_copy_bandwidth", c_double, P, c_size_t, c_int)
_proto("cugraph_type_erased_device_array_release", P, P)
# multi-GPU communicator contexts (include/cugraph_amd/comm.h)
_proto("cugraph_amd_comm_unique_id_size", c_size_t)
_proto("cugraph_amd_comm_get_unique_id", c_int, P, PP)
_proto("cugraph_amd_mg_context_create_rccl", c_int, P, c_int, c_int, c_int, PP, PP)
_proto("cugraph_amd_mg_context_create_ops", c_int, P, P, P, c_int, PP, PP)
_proto("cugraph_amd_mg_context_free", None, P)


def assert_success(code, err, api_name):
    """utils.pyx:37-80: map error codes to Python exceptions."""
    if code == 0:
        return
    msg = lib.cugraph_error_message(err) if err else b""
    msg = msg.decode() if isinstance(msg, bytes) else str(msg)
    if err:
        lib.cugraph_error_free(err)
    code_str = CODES.get(code, str(code))
    text = f"non-success value returned from {api_name}: {code_str} {msg}"
    if code in (2, 4):
        raise ValueError(text)
    if code == 3:
        raise MemoryError(text)
    if code == 5:
        raise NotImplementedError(text)
    if code == 6:
        raise TypeError(text)
    raise RuntimeError(text)


def call(api_name, *args):
    """Call an entry point whose last argument is ``cugraph_error_t**``."""
    err = ctypes.c_void_p()
    code = getattr(lib, api_name)(*args, ctypes.byref(err))
    assert_success(code, err.value, api_name)

"""pylibcugraph-compatible Python surface over the MI355X libcugraph_c.

Mirrors the reference's Cython shim (``python/pylibcugraph/pylibcugraph``) for the
hot path: ``ResourceHandle`` (resource_handle.pyx:25-46), ``GraphProperties``
(graph_properties.pyx:17-35), ``SGGraph``/``MGGraph`` (graphs.pyx:60-330),
``pagerank`` (pagerank.pyx:57-224), ``personalized_pagerank``
(personalized_pagerank.pyx), ``bfs`` (bfs.pyx:59-200), ``sssp`` (sssp.pyx:52-178),
``louvain`` (louvain.pyx:58-149) -- same argument names, order, return tuples and
exception types.  Arrays come back as GPU torch tensors (the reference returns
cupy arrays).
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._arrays import (DeviceArray, DeviceView, copy_view_to_tensor, copy_views_to_tensors, optional_view,
                      to_device_tensor, views_to_tensors_owned, vptr)

from . import generators  # noqa: E402,F401  (MI355X build extensions)
from . import comms  # noqa: E402,F401  (multi-GPU communicator contexts)

__all__ = ["trim_device_cache", "ResourceHandle", "GraphProperties", "SGGraph", "MGGraph", "pagerank",
           "personalized_pagerank", "katz_centrality", "eigenvector_centrality", "hits", "bfs", "sssp",
           "louvain", "version"]


def allocator_stats():
    """libcugraph_c's caching allocator counters: dict of driver allocations, their
    bytes and seconds, out-of-memory trims and the bytes cached now."""
    out = (ctypes.c_double * 5)()
    _lib.lib.cugraph_amd_allocator_stats(out)
    return {"mallocs": int(out[0]), "malloc_bytes": int(out[1]), "malloc_s": out[2], "oom_trims": int(out[3]),
            "cached_bytes": int(out[4])}


def trim_device_cache():
    """Return libcugraph_c's cached HBM blocks to the driver (ext.h
    cugraph_amd_trim_device_cache); call it beside torch.cuda.empty_cache().
    Returns the bytes released."""
    return int(_lib.lib.cugraph_amd_trim_device_cache())


def version():
    return _lib.lib.cugraph_amd_version().decode()


class ResourceHandle:
    """resource_handle.pyx:25-46.  ``handle`` may be a communicator pointer
    (``cugraph.dask.comms``) for multi-GPU use, else None."""

    def __init__(self, handle=None):
        p = None if handle is None else ctypes.c_void_p(int(handle))
        self.c_resource_handle_ptr = _lib.lib.cugraph_create_resource_handle(p)
        if not self.c_resource_handle_ptr:
            raise RuntimeError("cugraph_create_resource_handle failed")

    @property
    def ptr(self):
        return self.c_resource_handle_ptr

    def get_rank(self):
        return _lib.lib.cugraph_resource_handle_get_rank(self.c_resource_handle_ptr)

    # measurement hooks (include/cugraph_amd/ext.h)
    def set_profiling(self, enable=True):
        _lib.lib.cugraph_amd_set_profiling(self.c_resource_handle_ptr, 1 if enable else 0)

    def set_option(self, name, value):
        """Measurement / A-B switch of the kernels (cugraph_amd_set_option); ``None``
        or "defaults" restores the production settings."""
        if name is None:
            name, value = "defaults", 0
        _lib.call("cugraph_amd_set_option", self.c_resource_handle_ptr, name.encode(), float(value))

    def last_iterations(self):
        return _lib.lib.cugraph_amd_last_iterations(self.c_resource_handle_ptr)

    def last_hot_kernel_ms(self):
        return _lib.lib.cugraph_amd_last_hot_kernel_ms(self.c_resource_handle_ptr)

    def last_hot_kernel_launches(self):
        return _lib.lib.cugraph_amd_last_hot_kernel_launches(self.c_resource_handle_ptr)

    def last_bfs_levels(self):
        return _lib.lib.cugraph_amd_last_bfs_levels(self.c_resource_handle_ptr)

    def last_bfs_bottom_up_steps(self):
        return _lib.lib.cugraph_amd_last_bfs_bottom_up_steps(self.c_resource_handle_ptr)

    def last_louvain_levels(self):
        return _lib.lib.cugraph_amd_last_louvain_levels(self.c_resource_handle_ptr)

    def last_louvain_sweep_bytes(self):
        """Multi-GPU Louvain: average bytes this rank sent per local-move sweep."""
        return _lib.lib.cugraph_amd_last_louvain_sweep_bytes(self.c_resource_handle_ptr)

    def last_louvain_partition(self):
        """Multi-GPU Louvain: (level-0 edges, level-0 ghosts) of this rank's 1D share."""
        e, g = ctypes.c_int64(), ctypes.c_int64()
        _lib.lib.cugraph_amd_last_louvain_partition(self.c_resource_handle_ptr, ctypes.byref(e), ctypes.byref(g))
        return e.value, g.value

    def measure_copy_bandwidth(self, nbytes=4 << 30, reps=10):
        """HBM ceiling: 16-B-per-lane copy kernel on this handle's stream, GB/s (read + write)."""
        r = _lib.lib.cugraph_amd_measure_copy_bandwidth(self.c_resource_handle_ptr, int(nbytes), int(reps))
        if r < 0:
            raise RuntimeError("cugraph_amd_measure_copy_bandwidth failed")
        return r

    def __del__(self, _sd=_lib.SHUTDOWN, _free=_lib.lib.cugraph_free_resource_handle):
        p = getattr(self, "c_resource_handle_ptr", None)
        if p and not _sd[0]:
            _free(p)
            self.c_resource_handle_ptr = None


class GraphProperties:
    """graph_properties.pyx:17-35."""

    def __init__(self, is_symmetric=False, is_multigraph=False):
        self.is_symmetric = bool(is_symmetric)
        self.is_multigraph = bool(is_multigraph)

    def _c(self):
        return _lib.GraphPropertiesStruct(int(self.is_symmetric), int(self.is_multigraph))

    def __getnewargs_ex__(self):
        return ((), {"is_symmetric": self.is_symmetric, "is_multigraph": self.is_multigraph})


class _GPUGraph:
    c_graph_ptr = None

    def number_of_vertices(self):
        return _lib.lib.cugraph_amd_graph_get_number_of_vertices(self.c_graph_ptr)

    def number_of_edges(self):
        return _lib.lib.cugraph_amd_graph_get_number_of_edges(self.c_graph_ptr)

    def adjacency(self, resource_handle, transposed=False):
        """(offsets, indices, weights|None) in internal ids (MI355X build extension)."""
        o, i, w = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        _lib.call("cugraph_amd_graph_get_adjacency", resource_handle.ptr, self.c_graph_ptr,
                  1 if transposed else 0, ctypes.byref(o), ctypes.byref(i), ctypes.byref(w))
        h = resource_handle.ptr
        out = (DeviceArray(o.value).to_tensor(h), DeviceArray(i.value).to_tensor(h),
               DeviceArray(w.value).to_tensor(h) if w.value else None)
        return out

    def out_weight_sums(self, resource_handle):
        """Per-vertex out-weight sums in internal order (weight dtype; out-degrees when
        unweighted), as PageRank computes them (MI355X build extension)."""
        a = ctypes.c_void_p()
        _lib.call("cugraph_amd_graph_get_out_weight_sums", resource_handle.ptr, self.c_graph_ptr, ctypes.byref(a))
        return DeviceArray(a.value).to_tensor(resource_handle.ptr)


def _check_bool(name, v):
    if not isinstance(v, (int, bool)):
        raise TypeError(f"expected int or bool for {name}, got {type(v)}")


class SGGraph(_GPUGraph):
    """graphs.pyx:60-240."""

    def __init__(self, resource_handle, graph_properties, src_array, dst_array, weight_array,
                 store_transposed=False, renumber=False, do_expensive_check=False,
                 edge_id_array=None, edge_type_array=None):
        _check_bool("store_transposed", store_transposed)
        _check_bool("renumber", renumber)
        _check_bool("do_expensive_check", do_expensive_check)
        if edge_id_array is not None or edge_type_array is not None:
            raise NotImplementedError("edge ids / edge types are not supported by this build")
        src = DeviceView(src_array)
        dst = DeviceView(dst_array)
        if dst.c_type != src.c_type:
            dst = DeviceView(dst.tensor.to(src.tensor.dtype))
        wgt = optional_view(weight_array)
        props = graph_properties._c()
        g = ctypes.c_void_p()
        _lib.call("cugraph_sg_graph_create", resource_handle.ptr, ctypes.byref(props), src.ptr, dst.ptr,
                  vptr(wgt), None, None, int(bool(store_transposed)), int(bool(renumber)),
                  int(bool(do_expensive_check)), ctypes.byref(g))
        self.c_graph_ptr = g.value
        self._mg = False

    def __del__(self, _sd=_lib.SHUTDOWN, _free=_lib.lib.cugraph_sg_graph_free):
        if getattr(self, "c_graph_ptr", None) and not _sd[0]:
            _free(self.c_graph_ptr)
            self.c_graph_ptr = None


class MGGraph(_GPUGraph):
    """graphs.pyx:247-330: collective over the communicator in the handle."""

    def __init__(self, resource_handle, graph_properties, src_array, dst_array, weight_array,
                 store_transposed=False, num_edges=-1, do_expensive_check=False,
                 edge_id_array=None, edge_type_array=None):
        _check_bool("store_transposed", store_transposed)
        src = DeviceView(src_array)
        dst = DeviceView(dst_array, src.tensor.dtype)
        wgt = optional_view(weight_array)
        if num_edges < 0:
            raise ValueError("num_edges (global edge count) is required for MGGraph")
        props = graph_properties._c()
        g = ctypes.c_void_p()
        _lib.call("cugraph_mg_graph_create", resource_handle.ptr, ctypes.byref(props), src.ptr, dst.ptr,
                  vptr(wgt), None, None, int(bool(store_transposed)), int(num_edges),
                  int(bool(do_expensive_check)), ctypes.byref(g))
        self.c_graph_ptr = g.value
        self._mg = True

    def __del__(self, _sd=_lib.SHUTDOWN, _free=_lib.lib.cugraph_mg_graph_free):
        if getattr(self, "c_graph_ptr", None) and not _sd[0]:
            _free(self.c_graph_ptr)
            self.c_graph_ptr = None


def _centrality(api, resource_handle, graph, *views_and_scalars):
    res = ctypes.c_void_p()
    _lib.call(api, resource_handle.ptr, graph.c_graph_ptr, *views_and_scalars, ctypes.byref(res))
    v, x = views_to_tensors_owned(resource_handle.ptr, [_lib.lib.cugraph_centrality_result_get_vertices(res),
                                                        _lib.lib.cugraph_centrality_result_get_values(res)],
                                  res, _lib.lib.cugraph_centrality_result_free)
    return v, x


def pagerank(resource_handle, graph, precomputed_vertex_out_weight_vertices,
             precomputed_vertex_out_weight_sums, initial_guess_vertices, initial_guess_values,
             alpha, epsilon, max_iterations, do_expensive_check):
    """pagerank.pyx:57-224.  Returns (vertices, pageranks)."""
    a = optional_view(precomputed_vertex_out_weight_vertices)
    b = optional_view(precomputed_vertex_out_weight_sums)
    c = optional_view(initial_guess_vertices)
    d = optional_view(initial_guess_values)
    return _centrality("cugraph_pagerank", resource_handle, graph, vptr(a), vptr(b), vptr(c), vptr(d),
                       float(alpha), float(epsilon), int(max_iterations), int(bool(do_expensive_check)))


def personalized_pagerank(resource_handle, graph, precomputed_vertex_out_weight_vertices,
                          precomputed_vertex_out_weight_sums, initial_guess_vertices,
                          initial_guess_values, personalization_vertices, personalization_values,
                          alpha, epsilon, max_iterations, do_expensive_check):
    """personalized_pagerank.pyx.  Returns (vertices, pageranks)."""
    a = optional_view(precomputed_vertex_out_weight_vertices)
    b = optional_view(precomputed_vertex_out_weight_sums)
    c = optional_view(initial_guess_vertices)
    d = optional_view(initial_guess_values)
    e = optional_view(personalization_vertices)
    f = optional_view(personalization_values)
    return _centrality("cugraph_personalized_pagerank", resource_handle, graph, vptr(a), vptr(b), vptr(c),
                       vptr(d), vptr(e), vptr(f), float(alpha), float(epsilon), int(max_iterations),
                       int(bool(do_expensive_check)))


def _paths(resource_handle, res):
    v, d, p = views_to_tensors_owned(resource_handle.ptr, [_lib.lib.cugraph_paths_result_get_vertices(res),
                                                           _lib.lib.cugraph_paths_result_get_distances(res),
                                                           _lib.lib.cugraph_paths_result_get_predecessors(res)],
                                     res, _lib.lib.cugraph_paths_result_free)
    return v, d, p


def katz_centrality(resource_handle, graph, betas, alpha, beta, epsilon, max_iterations, do_expensive_check):
    """katz_centrality.pyx:57-155.  betas (optional) indexed by external vertex id.
    Returns (vertices, values)."""
    b = optional_view(betas)
    return _centrality("cugraph_katz_centrality", resource_handle, graph, vptr(b), float(alpha), float(beta),
                       float(epsilon), int(max_iterations), int(bool(do_expensive_check)))


def eigenvector_centrality(resource_handle, graph, epsilon, max_iterations, do_expensive_check):
    """eigenvector_centrality.pyx:57-136.  Returns (vertices, values)."""
    return _centrality("cugraph_eigenvector_centrality", resource_handle, graph, float(epsilon),
                       int(max_iterations), int(bool(do_expensive_check)))


def hits(resource_handle, graph, tol, max_iter, initial_hubs_guess_vertices, initial_hubs_guess_values,
         normalized, do_expensive_check):
    """hits.pyx:58-193.  Returns (vertices, hubs, authorities)."""
    gv = optional_view(initial_hubs_guess_vertices)
    gs = optional_view(initial_hubs_guess_values)
    res = ctypes.c_void_p()
    _lib.call("cugraph_hits", resource_handle.ptr, graph.c_graph_ptr, float(tol), int(max_iter), vptr(gv), vptr(gs),
              int(bool(normalized)), int(bool(do_expensive_check)), ctypes.byref(res))
    h = resource_handle.ptr
    try:
        v = copy_view_to_tensor(h, _lib.lib.cugraph_hits_result_get_vertices(res))
        hb = copy_view_to_tensor(h, _lib.lib.cugraph_hits_result_get_hubs(res))
        au = copy_view_to_tensor(h, _lib.lib.cugraph_hits_result_get_authorities(res))
        resource_handle._last_hits = (_lib.lib.cugraph_hits_result_get_hub_score_differences(res),
                                      _lib.lib.cugraph_hits_result_get_number_of_iterations(res))
    finally:
        _lib.lib.cugraph_hits_result_free(res)
    return v, hb, au


def bfs(handle, graph, sources, direction_optimizing, depth_limit, compute_predecessors,
        do_expensive_check):
    """bfs.pyx:59-200.  depth_limit <= 0 means unlimited (bfs.pyx:148-149).
    Returns (distances, predecessors, vertices)."""
    # the library renumbers sources in place (bfs.cpp:96-114): hand it a private copy
    src = DeviceView(to_device_tensor(sources).clone())
    if depth_limit is None or depth_limit <= 0:
        depth_limit = 2 ** 31 - 2
    res = ctypes.c_void_p()
    _lib.call("cugraph_bfs", handle.ptr, graph.c_graph_ptr, src.ptr, int(bool(direction_optimizing)),
              int(depth_limit), int(bool(compute_predecessors)), int(bool(do_expensive_check)),
              ctypes.byref(res))
    v, d, p = _paths(handle, res)
    return d, p, v


def bfs_paths(resource_handle, graph, sources, destinations, depth_limit=0):
    """BFS (predecessors on) followed by ``cugraph_extract_paths`` on its result
    (reference traversal/extract_bfs_paths_impl.cuh; the reference declares the C
    entry in _cugraph_c/algorithms.pxd without a Python wrapper).  Returns
    (paths [len(destinations) x max_path_length] tensor, max_path_length)."""
    src = DeviceView(to_device_tensor(sources).clone())
    dst = DeviceView(to_device_tensor(destinations), src.tensor.dtype)
    if depth_limit is None or depth_limit <= 0:
        depth_limit = 2 ** 31 - 2
    res = ctypes.c_void_p()
    _lib.call("cugraph_bfs", resource_handle.ptr, graph.c_graph_ptr, src.ptr, 0, int(depth_limit), 1, 0,
              ctypes.byref(res))
    ep = ctypes.c_void_p()
    try:
        _lib.call("cugraph_extract_paths", resource_handle.ptr, graph.c_graph_ptr, src.ptr, res, dst.ptr,
                  ctypes.byref(ep))
    finally:
        _lib.lib.cugraph_paths_result_free(res)
    try:
        L = _lib.lib.cugraph_extract_paths_result_get_max_path_length(ep)
        paths = copy_view_to_tensor(resource_handle.ptr, _lib.lib.cugraph_extract_paths_result_get_paths(ep))
    finally:
        _lib.lib.cugraph_extract_paths_result_free(ep)
    return paths.reshape(-1, L) if L else paths, L


def sssp(resource_handle, graph, source, cutoff, compute_predecessors, do_expensive_check):
    """sssp.pyx:52-178.  Returns (vertices, distances, predecessors)."""
    res = ctypes.c_void_p()
    _lib.call("cugraph_sssp", resource_handle.ptr, graph.c_graph_ptr, int(source), float(cutoff),
              int(bool(compute_predecessors)), int(bool(do_expensive_check)), ctypes.byref(res))
    return _paths(resource_handle, res)


def louvain(resource_handle, graph, max_level, resolution, do_expensive_check):
    """louvain.pyx:58-149.  Returns (vertices, clusters, modularity)."""
    res = ctypes.c_void_p()
    _lib.call("cugraph_louvain", resource_handle.ptr, graph.c_graph_ptr, int(max_level), float(resolution),
              int(bool(do_expensive_check)), ctypes.byref(res))
    h = resource_handle.ptr
    try:
        v = copy_view_to_tensor(h, _lib.lib.cugraph_heirarchical_clustering_result_get_vertices(res))
        c = copy_view_to_tensor(h, _lib.lib.cugraph_heirarchical_clustering_result_get_clusters(res))
        q = _lib.lib.cugraph_heirarchical_clustering_result_get_modularity(res)
    finally:
        _lib.lib.cugraph_heirarchical_clustering_result_free(res)
    return v, c, q


def louvain_dendrogram(resource_handle, graph, max_level, resolution, do_expensive_check=False):
    """Extension (the reference C++ ``cugraph::louvain`` returns the Dendrogram,
    louvain_impl.cuh:280-301).  Returns (vertices, clusters, modularity, levels):
    ``levels[i]`` is this rank's slice of dendrogram level i (its level-i vertices
    in global-id order; values are level-(i+1) ids)."""
    res = ctypes.c_void_p()
    _lib.call("cugraph_louvain", resource_handle.ptr, graph.c_graph_ptr, int(max_level), float(resolution),
              int(bool(do_expensive_check)), ctypes.byref(res))
    h = resource_handle.ptr
    try:
        v = copy_view_to_tensor(h, _lib.lib.cugraph_heirarchical_clustering_result_get_vertices(res))
        c = copy_view_to_tensor(h, _lib.lib.cugraph_heirarchical_clustering_result_get_clusters(res))
        q = _lib.lib.cugraph_heirarchical_clustering_result_get_modularity(res)
        n = _lib.lib.cugraph_amd_heirarchical_clustering_result_get_num_levels(res)
        levels = [copy_view_to_tensor(h, _lib.lib.cugraph_amd_heirarchical_clustering_result_get_level(res, i))
                  for i in range(n)]
    finally:
        _lib.lib.cugraph_heirarchical_clustering_result_free(res)
    return v, c, q, levels

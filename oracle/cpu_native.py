"""ctypes loader for the compiled CPU restatements (oracle/cpu_baseline.c,
oracle/cpu_louvain.c, oracle/cpu_sssp.c).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): bench.py's cpu_baseline leg
times it as the secondary CPU baseline of SURVEY.md §8d.  Built by
``make -C oracle`` (``__graft_entry__.build()`` runs it).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libcpu_baseline.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise FileNotFoundError(f"{_LIB} not built (make -C oracle)")
        _lib = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        _lib.cpu_pagerank.restype = ctypes.c_double
        _lib.cpu_pagerank.argtypes = [P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_int, P]
        _lib.cpu_pagerank_f64.restype = ctypes.c_int
        _lib.cpu_pagerank_f64.argtypes = [P, P, ctypes.c_int64, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                          ctypes.c_int, P]
        _lib.cpu_bfs.restype = ctypes.c_double
        _lib.cpu_bfs.argtypes = [P, P, ctypes.c_int64, ctypes.c_int32, ctypes.c_int, P, P]
        for f in (_lib.cpu_sssp_f32, _lib.cpu_sssp_f64):
            f.restype = ctypes.c_int
            f.argtypes = [P, P, P, ctypes.c_int64, ctypes.c_int32, ctypes.c_double, P, P,
                          ctypes.POINTER(ctypes.c_double)]
        _lib.cpu_louvain.restype = ctypes.c_int
        _lib.cpu_louvain.argtypes = [ctypes.c_int64, P, P, P, ctypes.c_int, ctypes.c_double, ctypes.c_int, P, P, P]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def pagerank(offsets, indices, iterations, alpha=0.85, threads=1):
    """Time `iterations` reference power iterations on the CSC (offsets int64,
    indices int32).  Returns (seconds, pageranks float32)."""
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    idx = np.ascontiguousarray(indices, dtype=np.int32)
    nv = off.size - 1
    pr = np.empty(nv, dtype=np.float32)
    t = lib().cpu_pagerank(_p(off), _p(idx), nv, int(iterations), float(alpha), int(threads), _p(pr))
    if t < 0:
        raise MemoryError("cpu_pagerank allocation failed")
    return t, pr


def bfs(offsets, indices, source, threads=1):
    """Time one BFS on the CSR.  Returns (seconds, distances, predecessors)."""
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    idx = np.ascontiguousarray(indices, dtype=np.int32)
    nv = off.size - 1
    dist = np.empty(nv, dtype=np.int32)
    pred = np.empty(nv, dtype=np.int32)
    t = lib().cpu_bfs(_p(off), _p(idx), nv, int(source), int(threads), _p(dist), _p(pred))
    if t < 0:
        raise MemoryError("cpu_bfs allocation failed")
    return t, dist, pred


def pagerank_f64(offsets, indices, alpha=0.85, epsilon=1e-6, max_iterations=500, threads=0):
    """The fp64 oracle PageRank (oracle/pagerank.py semantics) on a CSC, compiled
    with OpenMP (threads=0: the OpenMP default).  Returns (ranks float64, iterations)."""
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    idx = np.ascontiguousarray(indices, dtype=np.int32)
    nv = off.size - 1
    pr = np.empty(nv, dtype=np.float64)
    it = lib().cpu_pagerank_f64(_p(off), _p(idx), nv, float(alpha), float(epsilon), int(max_iterations),
                                int(threads), _p(pr))
    if it == -2:
        raise MemoryError("cpu_pagerank_f64 allocation failed")
    if it == -1:
        raise RuntimeError("PageRank failed to converge.")
    return pr, it


def louvain(offsets, indices, weights, max_level=100, resolution=1.0, threads=0):
    """The oracle Louvain (oracle/louvain.py semantics) on a CSR in internal ids,
    compiled with OpenMP.  Returns (clustering int64[V], modularity, levels)."""
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    idx = np.ascontiguousarray(indices, dtype=np.int32)
    w = np.ascontiguousarray(weights, dtype=np.float64)
    nv = off.size - 1
    c = np.empty(max(nv, 1), dtype=np.int64)
    q = ctypes.c_double(0.0)
    lv = ctypes.c_int(0)
    rc = lib().cpu_louvain(nv, _p(off), _p(idx), _p(w), int(max_level), float(resolution), int(threads), _p(c),
                           ctypes.byref(q), ctypes.byref(lv))
    if rc == -2:
        raise MemoryError("cpu_louvain allocation failed")
    return c[:nv], q.value, lv.value


def sssp(offsets, indices, weights, source, cutoff=float("inf")):
    """Near-far SSSP (oracle/cpu_sssp.c: sssp_impl.cuh:79-270 restated, one thread)
    on a CSR in internal ids; weights float32 or float64 pick the weight type.
    Returns (seconds, distances, predecessors int32 (-1: none), rounds)."""
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    idx = np.ascontiguousarray(indices, dtype=np.int32)
    w = np.ascontiguousarray(weights)
    if w.dtype not in (np.float32, np.float64):
        w = w.astype(np.float32)
    nv = off.size - 1
    dist = np.empty(nv, dtype=w.dtype)
    pred = np.empty(nv, dtype=np.int32)
    t = ctypes.c_double(0.0)
    f = lib().cpu_sssp_f32 if w.dtype == np.float32 else lib().cpu_sssp_f64
    rounds = f(_p(off), _p(idx), _p(w), nv, int(source), float(cutoff), _p(dist), _p(pred), ctypes.byref(t))
    if rounds == -2:
        raise MemoryError("cpu_sssp allocation failed")
    return t.value, dist, pred, rounds

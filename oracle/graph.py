"""Oracle graph construction (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates how the reference turns an edge list into its CSR/CSC ``graph_t``:

* renumbering -- ``cpp/src/structure/renumber_edgelist_impl.cuh:95-452``
  (``compute_renumber_map``): the vertex set is the sorted union of all edge
  endpoints (or the given vertex list), vertices are ordered by DESCENDING
  major degree with a stable sort (``:384-390``), so ties keep ascending
  external id; the number map is ``new id -> external id``.
* no renumbering -- ``create_graph_from_edgelist_impl.cuh:611-620``: the
  vertex count is ``max(src, dst) + 1`` and ids are used as is.
* compression -- ``structure/detail/structure_utils.cuh:162-232``: edges are
  grouped by major (src for CSR, dst for CSC) and each adjacency list is sorted
  by minor id (``sort_adjacency_list``); multi-edges are kept at the C ABI.
* ``cugraph.Graph`` preprocessing -- ``python/cugraph/cugraph/structure/
  symmetrize.py:78-93``: dedup keeping the MIN weight, symmetrise when
  undirected; ``graph_implementation/simpleGraph.py:840-843``: unweighted
  graphs get all-ones fp32 weights.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np


@dataclass
class Csr:
    """Compressed adjacency over internal ids 0..V-1 (major -> minors)."""

    num_vertices: int
    offsets: np.ndarray  # int64[V+1]
    indices: np.ndarray  # int64[E], internal ids, sorted within each row
    weights: Optional[np.ndarray]  # float64[E] or None (unweighted)
    number_map: np.ndarray  # int64[V]: internal id -> external id
    transposed: bool  # True: CSC (major = dst)

    @property
    def num_edges(self) -> int:
        return int(self.indices.shape[0])

    def degrees(self) -> np.ndarray:
        return np.diff(self.offsets)

    def majors(self) -> np.ndarray:
        return np.repeat(np.arange(self.num_vertices, dtype=np.int64), self.degrees())

    def coo(self):
        """(src, dst, w) in internal ids, whatever the storage orientation."""
        maj = self.majors()
        w = self.weights if self.weights is not None else np.ones(self.num_edges)
        if self.transposed:
            return self.indices.copy(), maj, w
        return maj, self.indices.copy(), w


def renumber_map(src, dst, store_transposed: bool, vertices=None) -> np.ndarray:
    """Number map (new id -> external id), renumber_edgelist_impl.cuh:95-452."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    if vertices is None:
        verts = np.unique(np.concatenate([src, dst]))
    else:
        verts = np.unique(np.asarray(vertices, dtype=np.int64))
    majors = dst if store_transposed else src
    pos = np.searchsorted(verts, majors)
    deg = np.bincount(pos, minlength=verts.shape[0]) if majors.size else np.zeros(verts.shape[0], np.int64)
    order = np.argsort(-deg, kind="stable")  # descending degree, ties by ascending id
    return verts[order]


def _pair_order(major, minor):
    """Stable order by (major, minor) -- np.lexsort((minor, major)), via one int64
    key when both fit 31 bits (much faster on 10^7+ edges)."""
    major = np.asarray(major, dtype=np.int64)
    minor = np.asarray(minor, dtype=np.int64)
    if major.size and min(major.min(), minor.min()) >= 0 and max(major.max(), minor.max()) < (1 << 31):
        return np.argsort((major << 31) | minor, kind="stable")
    return np.lexsort((minor, major))


def compress(num_vertices, src_int, dst_int, w, store_transposed: bool):
    """CSR (or CSC) with sorted adjacency lists, structure_utils.cuh:162-232."""
    major = dst_int if store_transposed else src_int
    minor = src_int if store_transposed else dst_int
    perm = _pair_order(major, minor)  # stable; duplicates keep input order
    major = major[perm]
    minor = minor[perm]
    counts = np.bincount(major, minlength=num_vertices) if major.size else np.zeros(num_vertices, np.int64)
    offsets = np.zeros(num_vertices + 1, dtype=np.int64)
    np.cumsum(counts, out=offsets[1:])
    weights = None if w is None else np.asarray(w, dtype=np.float64)[perm]
    return offsets, minor.astype(np.int64), weights


def create_graph(src, dst, weights=None, store_transposed=False, renumber=True, vertices=None) -> Csr:
    """``cugraph_sg_graph_create`` restated (c_api/graph_sg.cpp:231 ->
    create_graph_from_edgelist_impl.cuh:557-776)."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    if renumber:
        nmap = renumber_map(src, dst, store_transposed, vertices)
        order = np.argsort(nmap, kind="stable")
        sorted_ext = nmap[order]
        src_i = order[np.searchsorted(sorted_ext, src)]
        dst_i = order[np.searchsorted(sorted_ext, dst)]
        nv = int(nmap.shape[0])
    else:
        if vertices is not None:
            nv = int(len(vertices))
        else:
            nv = int(max(src.max(initial=-1), dst.max(initial=-1)) + 1)
        nmap = np.arange(nv, dtype=np.int64)
        src_i, dst_i = src, dst
    offsets, indices, w = compress(nv, src_i, dst_i, weights, store_transposed)
    return Csr(nv, offsets, indices, w, nmap, store_transposed)


def transpose(g: Csr) -> Csr:
    """Same numbering, other orientation (c_api/graph.hpp:42-79 transpose_storage)."""
    s, d, w = g.coo()
    offsets, indices, wt = compress(g.num_vertices, s, d, None if g.weights is None else w, not g.transposed)
    return Csr(g.num_vertices, offsets, indices, wt, g.number_map.copy(), not g.transposed)


def symmetrize_dedup(src, dst, weights=None, symmetrize=True):
    """cugraph.Graph preprocessing (structure/symmetrize.py:78-93):
    concat reversed edges when undirected, then groupby([src,dst]).min()."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    w = None if weights is None else np.asarray(weights, dtype=np.float64)
    if symmetrize:
        src, dst = np.concatenate([src, dst]), np.concatenate([dst, src])
        if w is not None:
            w = np.concatenate([w, w])
    if src.size == 0:
        return src, dst, w
    perm = _pair_order(src, dst)
    s, d = src[perm], dst[perm]
    first = np.ones(s.shape[0], dtype=bool)
    first[1:] = (s[1:] != s[:-1]) | (d[1:] != d[:-1])
    if w is not None:
        ww = w[perm]
        wmin = np.minimum.reduceat(ww, np.flatnonzero(first))
        return s[first], d[first], wmin
    return s[first], d[first], None


def read_csv(path):
    """Space-delimited ``src dst [w]`` files of ``datasets/`` (as conftest.py:93-101)."""
    data = np.loadtxt(path, dtype=np.float64, ndmin=2)
    src = data[:, 0].astype(np.int64)
    dst = data[:, 1].astype(np.int64)
    w = data[:, 2].astype(np.float32).astype(np.float64) if data.shape[1] > 2 else None
    return src, dst, w

"""Oracle SSSP (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates ``detail::sssp`` of ``cpp/src/traversal/sssp_impl.cuh:79-270``:
distances start at ``numeric_limits<weight_t>::max()`` (0 at the source), a
relaxation ``new = dist[u] + w`` (in weight_t arithmetic) is pushed only when
``new < min(cutoff, dist[v])`` (e_op, ``:49-72``).  The near-far bucketing only
orders the work; the fixed point -- the minimum over paths of the left-folded
weight_t path sums, restricted to sums below ``cutoff`` -- is what we compute
here by frontier Bellman-Ford in the same precision.

Predecessors: the reference reduces pushes with ``reduce_op::minimum`` on the
(distance, predecessor) tuple (``:209``, ``prims/reduce_op.cuh:68-80``), so equal
distances pick the smaller predecessor within one push round.  Our build makes
the choice order-independent: the smallest internal id among all tight
in-neighbours (``dist[u] + w == dist[v]``), which matches every reference golden
vector (``cpp/tests/c_api/sssp_test.c:182-187``,
``python/pylibcugraph/pylibcugraph/tests/test_sssp.py``).
"""
from __future__ import annotations

import numpy as np


def sssp(num_vertices, offsets, indices, weights, source, cutoff=np.inf, dtype=np.float32, tie_key=None):
    V = int(num_vertices)
    offsets = np.asarray(offsets, dtype=np.int64)
    indices = np.asarray(indices, dtype=np.int64)
    w = np.asarray(weights).astype(dtype)
    big = np.finfo(dtype).max
    dist = np.full(V, big, dtype=dtype)
    pred = np.full(V, -1, dtype=np.int64)
    if V == 0:
        return dist, pred
    if not (0 <= source < V):
        raise ValueError("Invalid input argument: source vertex out-of-range.")
    dist[source] = 0
    cut = dtype(cutoff) if np.isfinite(cutoff) and cutoff < big else big
    frontier = np.array([source], dtype=np.int64)
    deg_all = np.diff(offsets)
    while frontier.size:
        deg = deg_all[frontier]
        tot = int(deg.sum())
        if tot == 0:
            break
        u = np.repeat(frontier, deg)
        start = np.repeat(offsets[frontier], deg)
        local = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(deg) - deg, deg)
        e = start + local
        v = indices[e]
        nd = (dist[u] + w[e]).astype(dtype)
        m = (nd < dist[v]) & (nd < cut)
        if not m.any():
            break
        v, nd = v[m], nd[m]
        before = dist.copy()
        np.minimum.at(dist, v, nd)
        frontier = np.nonzero(dist < before)[0]
    # predecessor: min tie-key over tight in-edges
    key = np.arange(V, dtype=np.int64) if tie_key is None else np.asarray(tie_key, dtype=np.int64)
    srcs = np.repeat(np.arange(V, dtype=np.int64), deg_all)
    reach = dist[srcs] < big
    s, d, ww = srcs[reach], indices[reach], w[reach]
    tight = ((dist[s] + ww).astype(dtype) == dist[d]) & (d != source)
    s, d = s[tight], d[tight]
    best = np.full(V, np.iinfo(np.int64).max, dtype=np.int64)
    np.minimum.at(best, d, key[s])
    has = best != np.iinfo(np.int64).max
    inv = np.empty(V, dtype=np.int64)
    inv[key] = np.arange(V, dtype=np.int64)
    pred[has] = inv[best[has]]
    return dist, pred

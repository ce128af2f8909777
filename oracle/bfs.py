"""Oracle BFS (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates ``detail::bfs`` of ``cpp/src/traversal/bfs_impl.cuh:94-287`` and the
CPU reference ``cpp/tests/traversal/bfs_test.cpp:41-79``: level-synchronous
expansion from every source at distance 0; a vertex first reached at level d
gets distance d+1; unreached vertices keep ``INT_MAX`` (``invalid_distance``,
``:150-157``) and predecessor -1; the loop stops when the frontier is empty or
``depth >= depth_limit`` (``:278-285``).

Predecessors: the reference picks whichever pusher wins an ``atomicOr``
(``bfs_impl.cuh:76-83``), i.e. any frontier neighbour.  Our build makes the
choice deterministic -- the frontier neighbour with the smallest *internal*
id -- which is also what the reference's C golden vector shows
(``cpp/tests/c_api/bfs_test.c:124-129``).  ``tie_key`` lets a test give the
internal numbering so the oracle reproduces that choice exactly.
"""
from __future__ import annotations

import numpy as np

INT32_MAX = np.iinfo(np.int32).max
INT64_MAX = np.iinfo(np.int64).max


def bfs(num_vertices, offsets, indices, sources, depth_limit=None, tie_key=None, invalid_distance=INT32_MAX):
    """CSR (out-edges) in one numbering.  Returns (distances int64, predecessors int64)."""
    V = int(num_vertices)
    offsets = np.asarray(offsets, dtype=np.int64)
    indices = np.asarray(indices, dtype=np.int64)
    dist = np.full(V, invalid_distance, dtype=np.int64)
    pred = np.full(V, -1, dtype=np.int64)
    key = np.arange(V, dtype=np.int64) if tie_key is None else np.asarray(tie_key, dtype=np.int64)
    src = np.unique(np.asarray(sources, dtype=np.int64))
    if V == 0 or src.size == 0:
        return dist, pred
    dist[src] = 0
    frontier = src
    depth = 0
    limit = np.iinfo(np.int64).max if depth_limit is None else int(depth_limit)
    while frontier.size and depth < limit:
        deg = offsets[frontier + 1] - offsets[frontier]
        tot = int(deg.sum())
        if tot == 0:
            break
        u = np.repeat(frontier, deg)
        start = np.repeat(offsets[frontier], deg)
        local = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(deg) - deg, deg)
        v = indices[start + local]
        m = dist[v] == invalid_distance
        u, v = u[m], v[m]
        if v.size == 0:
            break
        best = np.full(V, INT64_MAX, dtype=np.int64)
        np.minimum.at(best, v, key[u])
        nxt = np.unique(v)
        dist[nxt] = depth + 1
        # map the winning key back to a vertex id
        inv = np.empty(V, dtype=np.int64)
        inv[key] = np.arange(V, dtype=np.int64)
        pred[nxt] = inv[best[nxt]]
        frontier = nxt
        depth += 1
    return dist, pred


def check_predecessors(offsets, indices, dist, pred, sources, invalid_distance=INT32_MAX):
    """Validity rule of cpp/tests/traversal/bfs_test.cpp:210-230: for every reached
    non-source v, dist[pred[v]] + 1 == dist[v] and the edge pred[v] -> v exists."""
    offsets = np.asarray(offsets, dtype=np.int64)
    indices = np.asarray(indices, dtype=np.int64)
    srcset = set(int(s) for s in np.asarray(sources).ravel())
    bad = []
    for v in np.nonzero(dist != invalid_distance)[0]:
        p = int(pred[v])
        if int(v) in srcset:
            if p != -1:
                bad.append(int(v))
            continue
        if p < 0 or dist[p] + 1 != dist[v]:
            bad.append(int(v))
            continue
        row = indices[offsets[p]:offsets[p + 1]]
        if not np.any(row == v):
            bad.append(int(v))
    return bad

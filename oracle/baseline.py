"""CPU baselines timed by bench.py (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

The reference's CPU path for PageRank is NetworkX (``nx.pagerank`` ->
``_pagerank_scipy``, networkx 3.4.2): a scipy CSR matrix and the power
iteration ``x = alpha*(x@A + sum(x[dangling])*p) + (1-alpha)*p`` in float64,
single-threaded.  ``pagerank_scipy_iterations`` restates exactly that loop body
on an already-built CSR (graph construction excluded, as the GPU timing
excludes it), for a fixed number of iterations so the sample is bounded.
"""
from __future__ import annotations

import time

import numpy as np


def pagerank_scipy_iterations(offsets, indices, num_vertices, iterations=5, alpha=0.85):
    """Time `iterations` NetworkX-style power iterations on the pull CSR
    (row v lists in-neighbours u).  Returns (seconds, edges_per_second)."""
    import scipy.sparse as sp

    V = int(num_vertices)
    E = int(indices.shape[0])
    offsets = np.asarray(offsets, dtype=np.int64)
    indices = np.asarray(indices, dtype=np.int64)
    outdeg = np.bincount(indices, minlength=V).astype(np.float64)
    data = np.ones(E, dtype=np.float64)
    # row-stochastic A[u, v] = 1/outdeg(u) for u -> v, stored as its transpose (rows = v)
    AT = sp.csr_matrix((data / outdeg[indices], indices, offsets), shape=(V, V))
    x = np.full(V, 1.0 / V)
    p = np.full(V, 1.0 / V)
    dangling = np.nonzero(outdeg == 0)[0]
    t0 = time.perf_counter()
    for _ in range(iterations):
        x = alpha * (AT @ x + x[dangling].sum() * p) + (1 - alpha) * p
    t = time.perf_counter() - t0
    return t, E * iterations / t


def bfs_numpy(offsets, indices, source, max_levels=1 << 30):
    """Level-synchronous numpy BFS (oracle/bfs.py without predecessors).
    Returns (seconds, reached_edges)."""
    offsets = np.asarray(offsets, dtype=np.int64)
    indices = np.asarray(indices)
    V = offsets.shape[0] - 1
    dist = np.full(V, -1, dtype=np.int32)
    dist[source] = 0
    frontier = np.array([source], dtype=np.int64)
    t0 = time.perf_counter()
    depth = 0
    while frontier.size and depth < max_levels:
        deg = offsets[frontier + 1] - offsets[frontier]
        tot = int(deg.sum())
        if tot == 0:
            break
        start = np.repeat(offsets[frontier], deg)
        local = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(deg) - deg, deg)
        nb = indices[start + local]
        nb = nb[dist[nb] < 0]
        nb = np.unique(nb)
        dist[nb] = depth + 1
        frontier = nb.astype(np.int64)
        depth += 1
    t = time.perf_counter() - t0
    reached = dist >= 0
    edges = int((offsets[1:] - offsets[:-1])[reached].sum())
    return t, edges


def networkx_bfs(src, dst, source):
    """The reference's CPU path for BFS: ``nx.single_source_shortest_path_length``
    on an undirected ``nx.Graph`` (pure Python, 1 core).  Returns
    (build_seconds, bfs_seconds, undirected edges of the source's component)."""
    import networkx as nx

    t0 = time.perf_counter()
    G = nx.Graph()
    G.add_edges_from(zip(np.asarray(src).tolist(), np.asarray(dst).tolist()))
    t1 = time.perf_counter()
    lengths = nx.single_source_shortest_path_length(G, int(source))
    t2 = time.perf_counter()
    e_cc = sum(G.degree(v) for v in lengths) // 2
    return t1 - t0, t2 - t1, e_cc


def networkx_louvain(src, dst, weights, seed=42):
    """The reference's CPU path for Louvain: ``nx.community.louvain_communities``
    (resolution 1, the given seed) + ``nx.community.modularity``.
    Returns (build_seconds, louvain_seconds, modularity)."""
    import networkx as nx

    t0 = time.perf_counter()
    G = nx.Graph()
    G.add_weighted_edges_from(zip(np.asarray(src).tolist(), np.asarray(dst).tolist(),
                                  np.asarray(weights, dtype=np.float64).tolist()))
    t1 = time.perf_counter()
    comms = nx.community.louvain_communities(G, weight="weight", resolution=1.0, seed=seed)
    t2 = time.perf_counter()
    q = nx.community.modularity(G, comms, weight="weight")
    return t1 - t0, t2 - t1, q


def networkx_pagerank(scale, alpha=0.85, epsilon=1e-6, seed=42):
    """The reference's CPU path for PageRank itself: ``nx.pagerank`` on an
    undirected ``nx.Graph`` of the symmetrised R-MAT graph of `scale` (numpy twin of
    the device generator), to convergence.  NetworkX stops on L1 < N * tol
    (networkx/algorithms/link_analysis/pagerank_alg.py, _pagerank_scipy), so tol =
    epsilon / N gives the reference's L1 < epsilon rule.  The iteration count is
    that of the same loop (pagerank_scipy_iterations' body) run to the same rule.
    Returns (build_seconds, pagerank_seconds, stored_edges, iterations)."""
    import networkx as nx
    import scipy.sparse as sp

    from oracle import graph as og
    from oracle import rmat

    s, d = rmat.rmat(scale, 16 << scale, seed=seed)
    s, d, _ = og.symmetrize_dedup(s, d, None)
    t0 = time.perf_counter()
    G = nx.Graph()
    G.add_edges_from(zip(s.tolist(), d.tolist()))
    t1 = time.perf_counter()
    N = G.number_of_nodes()
    nx.pagerank(G, alpha=alpha, tol=epsilon / N, max_iter=500)
    t2 = time.perf_counter()
    # iterations of the same power loop to the same stopping rule
    ids, inv = np.unique(np.concatenate([s, d]), return_inverse=True)
    si, di = inv[: s.size], inv[s.size:]
    V = ids.size
    outdeg = np.bincount(si, minlength=V).astype(np.float64)
    AT = sp.csr_matrix((1.0 / outdeg[si], (di, si)), shape=(V, V))
    x = np.full(V, 1.0 / V)
    it = 0
    while it < 500:
        xl = x
        x = alpha * (AT @ xl) + (1 - alpha) / V  # no dangling vertices in a symmetric edge-list graph
        it += 1
        if np.abs(x - xl).sum() < N * (epsilon / N):
            break
    return t1 - t0, t2 - t1, int(s.size), it

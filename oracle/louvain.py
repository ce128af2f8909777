"""Oracle Louvain (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates ``detail::louvain`` (``cpp/src/community/louvain_impl.cuh:46-237``),
``flatten_dendrogram`` (``:239-255``) and the helpers of
``cpp/src/community/detail/common_methods.cuh``:

* per level: vertex weights k = out-weight sums; cluster keys = all vertex ids
  with weights k (``louvain_impl.cuh:91-103``); Q of the singleton clustering;
  ``while new_Q > cur_Q + 1e-4`` run one synchronous local-move sweep with the
  up/down restriction alternating (``:156-199``); the dendrogram level keeps the
  clustering only when Q improved; stop when ``cur_Q <= best`` (``:203``), else
  contract (``common_methods.cuh:172-198``).
* local move (``update_clustering_by_delta_modularity``, ``common_methods.cuh:200-356``):
  old-cluster sum excludes self loops, self loops are subtracted from the own
  cluster's aggregated sum (``:270-292``, ``:49-74``); the gain is
  ``2*((new_sum - old_sum)/m - gamma*(a_new*k - a_old*k + k*k)/m^2)``; a
  neighbour cluster that is not a key gets ``a_new = numeric_limits::max()``
  (``:331-346``); best = max gain, ties -> smaller cluster id (``:77-94``),
  reduced with init (-1, 0) (``prims/per_v_transform_reduce_dst_key_aggregated_outgoing_e.cuh:159-163,803-807``);
  move only if gain > 0 and the direction matches ``up_down`` (``:97-109``).
* cluster weights (``compute_cluster_keys_and_values``, ``:358-382``): sums of
  edge weights grouped by the source's cluster -- only clusters with out-edges
  become keys.
* modularity (``:121-170``): ``sum_internal/m - gamma*sum(a_c^2)/m^2``.
* contraction (``structure/coarsen_graph_impl.cuh:527-632``): relabel edges by
  cluster, sum parallel edges, build the coarse graph over the unique labels
  renumbered by descending out-degree (stable), relabel the level.

Arithmetic is float64 (the reference uses weight_t; the GPU build uses
float64 accumulators too, so decisions are identical whenever the exact sums
are representable, e.g. integer weights).
"""
from __future__ import annotations

import numpy as np

FLT_MAX = float(np.finfo(np.float32).max)


class _Level:
    def __init__(self, V, src, dst, w):
        self.V = int(V)
        self.src = np.asarray(src, dtype=np.int64)
        self.dst = np.asarray(dst, dtype=np.int64)
        self.w = np.asarray(w, dtype=np.float64)


def _cluster_weights(g: _Level, clusters):
    """compute_cluster_keys_and_values: (present mask, weights) indexed by cluster id."""
    a = np.zeros(g.V, dtype=np.float64)
    present = np.zeros(g.V, dtype=bool)
    if g.src.size:
        c = clusters[g.src]
        np.add.at(a, c, g.w)
        present[c] = True
    return present, a


def _modularity(g: _Level, clusters, present, a, m, resolution):
    sum_sq = float(np.sum(a[present] ** 2))
    internal = float(g.w[clusters[g.src] == clusters[g.dst]].sum()) if g.src.size else 0.0
    return internal / m - (resolution * sum_sq) / (m * m)


def _update(g: _Level, clusters, present, a, k, m, resolution, up_down):
    V = g.V
    src, dst, w = g.src, g.dst, g.w
    cs, cd = clusters[src], clusters[dst]
    selfloop = src == dst
    old_sum = np.zeros(V)
    subtract = np.zeros(V)
    np.add.at(subtract, src[selfloop], w[selfloop])
    same = (~selfloop) & (cs == cd)
    np.add.at(old_sum, src[same], w[same])
    a_old = a[clusters]
    if src.size == 0:
        return clusters.copy()
    # aggregate (u, cluster(v)) -> sum w
    order = np.lexsort((cd, src))
    su, sc, sw = src[order], cd[order], w[order]
    first = np.ones(su.shape[0], dtype=bool)
    first[1:] = (su[1:] != su[:-1]) | (sc[1:] != sc[:-1])
    starts = np.nonzero(first)[0]
    pu, pc = su[starts], sc[starts]
    psum = np.add.reduceat(sw, starts)
    psum = psum - np.where(clusters[pu] == pc, subtract[pu], 0.0)
    a_new = np.where(present[pc], a[pc], FLT_MAX)
    kk = k[pu]
    dq = 2.0 * (((psum - old_sum[pu]) / m) - resolution * (a_new * kk - a_old[pu] * kk + kk * kk) / (m * m))
    # best per vertex: max dq, ties -> smaller cluster id (pairs sorted by (u, c))
    best_dq = np.full(V, -np.inf)
    np.maximum.at(best_dq, pu, dq)
    is_best = dq == best_dq[pu]
    best_c = np.full(V, np.iinfo(np.int64).max, dtype=np.int64)
    np.minimum.at(best_c, pu[is_best], pc[is_best])
    new = clusters.copy()
    mv = best_dq > 0.0
    v = np.nonzero(mv)[0]
    cand = best_c[v]
    ok = (cand > clusters[v]) == up_down
    new[v[ok]] = cand[ok]
    return new


def _contract(g: _Level, labels):
    cs, cd = labels[g.src], labels[g.dst]
    if cs.size:
        order = np.lexsort((cd, cs))
        s, d, w = cs[order], cd[order], g.w[order]
        first = np.ones(s.shape[0], dtype=bool)
        first[1:] = (s[1:] != s[:-1]) | (d[1:] != d[:-1])
        starts = np.nonzero(first)[0]
        s, d, w = s[starts], d[starts], np.add.reduceat(w, starts)
    else:
        s, d, w = cs, cd, g.w
    uniq = np.unique(labels)
    pos = np.searchsorted(uniq, s)
    deg = np.bincount(pos, minlength=uniq.shape[0])
    nmap = uniq[np.argsort(-deg, kind="stable")]  # new id -> label
    new_of_label = np.empty(int(uniq.max()) + 1 if uniq.size else 0, dtype=np.int64)
    new_of_label[nmap] = np.arange(nmap.shape[0], dtype=np.int64)
    return _Level(nmap.shape[0], new_of_label[s], new_of_label[d], w), new_of_label[labels]


def louvain(num_vertices, src, dst, weights, max_level=100, resolution=1.0, return_trace=False):
    """COO of the CSR graph (internal ids).  Returns (clustering, modularity, levels)."""
    g = _Level(num_vertices, src, dst, weights)
    m = float(g.w.sum())
    dendrogram = []
    best = -1.0
    trace = []
    while len(dendrogram) < max_level:
        V = g.V
        level = np.arange(V, dtype=np.int64)
        dendrogram.append(level)
        k = np.zeros(V)
        np.add.at(k, g.src, g.w)
        present = np.ones(V, dtype=bool)
        a = k.copy()
        clusters = np.arange(V, dtype=np.int64)
        new_q = _modularity(g, clusters, present, a, m, resolution)
        cur_q = new_q - 1.0
        up_down = True
        while new_q > cur_q + 0.0001:
            cur_q = new_q
            clusters = _update(g, clusters, present, a, k, m, resolution, up_down)
            present, a = _cluster_weights(g, clusters)
            up_down = not up_down
            new_q = _modularity(g, clusters, present, a, m, resolution)
            trace.append((len(dendrogram), cur_q, new_q))
            if new_q > cur_q:
                level[:] = clusters
        if cur_q <= best:
            break
        best = cur_q
        g, relabeled = _contract(g, level)
        dendrogram[-1] = relabeled
    clustering = np.arange(int(num_vertices), dtype=np.int64)
    for lvl in dendrogram:
        clustering = lvl[clustering]
    out = (clustering, best, len(dendrogram))
    return out + (trace,) if return_trace else out


def modularity(src, dst, weights, clustering, resolution=1.0):
    """Plain modularity of a given partition (same formula as compute_modularity)."""
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    w = np.asarray(weights, dtype=np.float64)
    c = np.asarray(clustering, dtype=np.int64)
    m = w.sum()
    a = np.zeros(int(c.max()) + 1 if c.size else 0)
    np.add.at(a, c[src], w)
    internal = w[c[src] == c[dst]].sum()
    return internal / m - resolution * float((a ** 2).sum()) / (m * m)

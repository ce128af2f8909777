"""Oracle PageRank (TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py).

Restates ``detail::pagerank`` of ``cpp/src/link_analysis/pagerank_impl.cuh:48-293``
step for step, in float64 by default (``dtype=np.float32`` replays the
reference's own fp32 arithmetic order-insensitively):

* out-weight sums (``:158-164``) unless precomputed;
* init 1/V, or the initial guess normalised by its sum (``:168-183``);
* per iteration (``:209-292``): dangling sum of pr over vertices with zero
  out-weight; x~ = pr / outw (divisor 1 for dangling); unvarying part
  ``(dangling*alpha + 1 - alpha) / V`` (0 when personalised); pull SpMV
  ``pr[v] = unvarying + sum_{u->v} x~[u] * w * alpha``; personalised mass
  ``(dangling*alpha + 1-alpha) * value / sum(values)`` added at the
  personalisation vertices (``:259-276``); L1 difference; stop when
  ``diff < epsilon`` (plain epsilon, not V*epsilon, ``:287``), otherwise fail
  after ``max_iterations`` (``:289-290``).
"""
from __future__ import annotations

import numpy as np


class PageRankNotConverged(RuntimeError):
    pass


def pagerank(num_vertices, src, dst, weights=None, alpha=0.85, epsilon=1e-6, max_iterations=500,
             personalization_vertices=None, personalization_values=None,
             initial_guess=None, out_weight_sums=None, dtype=np.float64, return_iterations=False):
    """Inputs are COO in one vertex numbering [0, num_vertices)."""
    V = int(num_vertices)
    src = np.asarray(src, dtype=np.int64)
    dst = np.asarray(dst, dtype=np.int64)
    w = np.ones(src.shape[0], dtype=dtype) if weights is None else np.asarray(weights).astype(dtype)
    if V == 0:
        out = np.zeros(0, dtype=dtype)
        return (out, 0) if return_iterations else out
    if not (0.0 <= alpha <= 1.0):
        raise ValueError("Invalid input argument: alpha should be in [0.0, 1.0].")
    if epsilon < 0.0:
        raise ValueError("Invalid input argument: epsilon should be non-negative.")
    a = dtype(alpha)
    if out_weight_sums is None:
        outw = np.bincount(src, weights=w, minlength=V).astype(dtype)
    else:
        outw = np.asarray(out_weight_sums).astype(dtype)
    if initial_guess is not None:
        pr = np.asarray(initial_guess).astype(dtype)
        s = pr.sum(dtype=dtype)
        if not s > 0:
            raise ValueError("sum of the PageRank initial guess values should be positive.")
        pr = pr / s
    else:
        pr = np.full(V, dtype(1.0) / dtype(V), dtype=dtype)
    pers = personalization_vertices is not None and len(personalization_vertices) > 0
    if pers:
        pv = np.asarray(personalization_vertices, dtype=np.int64)
        pval = np.asarray(personalization_values).astype(dtype)
        psum = pval.sum(dtype=dtype)
        if not psum > 0:
            raise ValueError("sum of personalization values should be positive.")
    dangling_mask = outw == 0
    divisor = np.where(dangling_mask, dtype(1.0), outw)
    it = 0
    while True:
        old = pr
        dangling = pr[dangling_mask].sum(dtype=dtype)
        xt = (pr / divisor).astype(dtype)
        base = dtype(0.0) if pers else (dangling * a + dtype(1.0 - alpha)) / dtype(V)
        contrib = (xt[src] * w * a).astype(dtype)
        pr = (base + np.bincount(dst, weights=contrib, minlength=V)).astype(dtype)
        if pers:
            np.add.at(pr, pv, (dangling * a + dtype(1.0 - alpha)) * (pval / psum))
        diff = np.abs(pr - old).sum(dtype=dtype)
        it += 1
        if diff < epsilon:
            break
        if it >= max_iterations:
            raise PageRankNotConverged("PageRank failed to converge.")
    return (pr, it) if return_iterations else pr


def pagerank_from_graph(g, **kw):
    """Run on an oracle ``Csr`` (either orientation); returns values by internal id."""
    s, d, w = g.coo()
    return pagerank(g.num_vertices, s, d, None if g.weights is None else w, **kw)

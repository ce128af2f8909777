"""Oracle Katz / eigenvector centrality / HITS (TEST INFRASTRUCTURE ONLY -- see
oracle/__init__.py).  All three are power iterations on the same pull SpMV as
PageRank; restated from the reference:

* katz: ``cpp/src/centrality/katz_centrality_impl.cuh:41-150`` with the C-API
  settings of ``c_api/katz.cpp:95-130`` (no initial guess -> 0, always
  L2-normalised, betas indexed by external vertex id, missing ids -> 0).  Stop when
  the L1 difference < epsilon; else "Katz Centrality failed to converge.".
* eigenvector: ``centrality/eigenvector_centrality_impl.cuh:40-125``: start
  1/V, y = A^T x (weighted), x = y / ||y||_2, stop when L1 difference < V*epsilon;
  else "Eigenvector Centrality failed to converge.".
* hits: ``link_analysis/hits_impl.cuh:40-160``: hubs start 1/V (or the guess
  normalised by its sum), authorities = A^T hubs, hubs' = A authorities (edge
  weights ignored), both divided by their max, stop when sum|hubs' - hubs| <
  epsilon (iteration count = that iteration's index, max_iterations otherwise,
  no error), optional final division by the sums.

Arithmetic in float64; the graph is a CSC/CSR pair in one numbering (oracle/graph.py).
"""
from __future__ import annotations

import numpy as np


def _pull(n, src, dst, w, x):
    """y[v] = sum over edges u->v of w * x[u]."""
    y = np.zeros(n)
    np.add.at(y, dst, w * x[src])
    return y


def katz(num_vertices, src, dst, weights, alpha, beta, epsilon, max_iterations, betas=None, normalize=True):
    n = int(num_vertices)
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    w = np.ones(src.size) if weights is None else np.asarray(weights, np.float64)
    b = np.full(n, float(beta)) if betas is None else np.asarray(betas, np.float64)
    x = np.zeros(n)
    it = 0
    while True:
        new = alpha * _pull(n, src, dst, w, x) + b
        diff = np.abs(new - x).sum()
        x = new
        it += 1
        if diff < epsilon:
            break
        if it >= max_iterations:
            raise RuntimeError("Katz Centrality failed to converge.")
    if normalize:
        nrm = np.sqrt((x * x).sum())
        if not nrm > 0:
            raise RuntimeError("L2 norm of the computed Katz Centrality values should be positive.")
        x = x / nrm
    return x


def eigenvector_centrality(num_vertices, src, dst, weights, epsilon, max_iterations):
    n = int(num_vertices)
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    w = np.ones(src.size) if weights is None else np.asarray(weights, np.float64)
    x = np.full(n, 1.0 / n)
    it = 0
    while True:
        old = x
        y = _pull(n, src, dst, w, x)
        x = y / np.sqrt((y * y).sum())
        diff = np.abs(x - old).sum()
        it += 1
        if diff < n * epsilon:
            return x
        if it >= max_iterations:
            raise RuntimeError("Eigenvector Centrality failed to converge.")


def hits(num_vertices, src, dst, epsilon, max_iterations, initial_hubs=None, normalize=True):
    """Returns (hubs, authorities, diff_sum, iterations)."""
    n = int(num_vertices)
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    ones = np.ones(src.size)
    if initial_hubs is not None:
        hubs = np.asarray(initial_hubs, np.float64).copy()
        hubs = hubs / hubs.sum()
    else:
        hubs = np.full(n, 1.0 / n)
    diff = np.finfo(np.float64).max
    iters = max_iterations
    auth = np.zeros(n)
    for it in range(max_iterations):
        auth = _pull(n, src, dst, ones, hubs)
        new = _pull(n, dst, src, ones, auth)
        mh, ma = new.max(), auth.max()
        if not (mh > 0 and ma > 0):
            raise RuntimeError("Norm is required to be a positive value.")
        new = new / mh
        auth = auth / ma
        diff = np.abs(new - hubs).sum()
        hubs = new
        if diff < epsilon:
            iters = it
            break
    if normalize:
        hubs = hubs / hubs.sum()
        auth = auth / auth.sum()
    return hubs, auth, diff, iters

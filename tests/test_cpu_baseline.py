"""The compiled CPU restatements (oracle/cpu_baseline.c, bench.py's secondary CPU
baseline, oracle/cpu_louvain.c and oracle/cpu_sssp.c) agree with the numpy oracle:
PageRank iterates converge to the oracle's ranks, BFS distances are exact,
single-threaded and with OpenMP, Louvain gives the oracle's clustering, modularity
and levels, and near-far SSSP the oracle's distances and predecessors bit for bit."""
import numpy as np
import pytest

from conftest import dataset_path
from oracle import bfs as obfs
from oracle import louvain as olv
from oracle import graph as og
from oracle import pagerank as opr
from oracle import rmat

cpu = pytest.importorskip("oracle.cpu_native")


def _built():
    try:
        cpu.lib()
        return True
    except FileNotFoundError:
        return False


pytestmark = pytest.mark.skipif(not _built(), reason="make -C oracle not run")


@pytest.mark.parametrize("threads", [1, 4])
def test_pagerank_matches_oracle(threads):
    s, d, _ = og.read_csv(dataset_path("karate.csv"))
    s, d, _ = og.symmetrize_dedup(s, d, None)
    g = og.create_graph(s, d, None, store_transposed=True, renumber=False)
    _, pr = cpu.pagerank(g.offsets, g.indices, 100, alpha=0.85, threads=threads)
    ref = opr.pagerank(g.num_vertices, s, d, None, 0.85, 1e-10, 500)
    assert np.allclose(pr, ref, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("threads", [1, 4])
def test_bfs_matches_oracle(threads):
    s, d = rmat.rmat(11, 16 << 11, seed=42)
    s, d, _ = og.symmetrize_dedup(s, d, None)
    g = og.create_graph(s, d, None, renumber=True)
    src = 0
    _, dist, pred = cpu.bfs(g.offsets, g.indices, src, threads=threads)
    rd, _ = obfs.bfs(g.num_vertices, g.offsets, g.indices, [src])
    assert np.array_equal(dist, rd)
    reached = (dist != np.iinfo(np.int32).max) & (np.arange(dist.size) != src)
    # every predecessor is a neighbour one level up (bfs_test.cpp:210-230 rule)
    assert np.all(dist[pred[reached]] == dist[reached] - 1)


def test_pagerank_f64_equals_numpy_oracle():
    s, d = rmat.rmat(12, 16 << 12, seed=42)
    s, d, _ = og.symmetrize_dedup(s, d, None)
    g = og.create_graph(s, d, None, store_transposed=True, renumber=True)
    ref, it_ref = opr.pagerank_from_graph(g, alpha=0.85, epsilon=1e-6, max_iterations=500, return_iterations=True)
    pr, it = cpu.pagerank_f64(g.offsets, g.indices, 0.85, 1e-6, 500, threads=4)
    assert it == it_ref
    assert np.max(np.abs(pr - ref) / ref) < 1e-12


@pytest.mark.parametrize("case", ["karate", "rmat10_int", "rmat12_int", "rmat12_frac", "rmat11_int_selfloops"])
@pytest.mark.parametrize("threads", [1, 4])
def test_louvain_matches_oracle(case, threads):
    """Integer weights: every sum is exact, so clustering, Q and level count are the
    numpy oracle's bit for bit; fractional weights: sums in another order, Q within
    1e-12 relative."""
    if case == "karate":
        s, d, w = og.read_csv(dataset_path("karate.csv"))
        s, d, w = og.symmetrize_dedup(s, d, np.asarray(w, np.float64))
    else:
        scale = int(case[4:6])
        s, d = rmat.rmat(scale, 16 << scale, seed=7)
        w = rmat.rmat_weights(s.size, seed=8).astype(np.float64)
        if "int" in case:
            w = np.floor(w * 8.0) + 1.0
        s, d, w = og.symmetrize_dedup(s, d, w)
        if "selfloops" not in case:
            keep = s != d
            s, d, w = s[keep], d[keep], w[keep]
    G = og.create_graph(s, d, w, renumber=True)
    oc, oq, olevels = olv.louvain(G.num_vertices, *G.coo())
    c, q, levels = cpu.louvain(G.offsets, G.indices, G.weights, threads=threads)
    if case == "rmat12_frac":
        assert abs(q - oq) <= 1e-12 * abs(oq)
    else:
        assert np.array_equal(c, oc) and q == oq and levels == olevels


@pytest.mark.parametrize("scale,symmetric,wdtype,cutoff", [(11, True, np.float32, np.inf), (12, False, np.float32, np.inf),
                                                          (11, True, np.float64, np.inf), (11, True, np.float32, 0.05)])
def test_sssp_matches_oracle(scale, symmetric, wdtype, cutoff):
    from oracle import sssp as osssp
    s, d = rmat.rmat(scale, 16 << scale, seed=42)
    w = rmat.rmat_weights(s.size, seed=43).astype(np.float64)
    s, d, w = og.symmetrize_dedup(s, d, w, symmetrize=symmetric)
    g = og.create_graph(s, d, w.astype(wdtype), renumber=True)
    for src in (0, g.num_vertices // 3):
        rd, rp = osssp.sssp(g.num_vertices, g.offsets, g.indices, g.weights, src, cutoff=cutoff, dtype=wdtype)
        _, dist, pred, rounds = cpu.sssp(g.offsets, g.indices, g.weights.astype(wdtype), src, cutoff)
        assert dist.dtype == wdtype and rounds > 0
        assert np.array_equal(dist, rd)
        assert np.array_equal(pred.astype(np.int64), rp)


def test_sssp_c_golden(golden):
    """cpp/tests/c_api/sssp_test.c:178-230 through the compiled restatement."""
    g = golden["sssp_c"]
    G = og.create_graph(g["src"], g["dst"], np.asarray(g["w"], np.float32), renumber=False)
    _, dist, pred, _ = cpu.sssp(G.offsets, G.indices, G.weights.astype(np.float32), g["source"], g["cutoff"])
    assert np.allclose(dist, np.asarray(g["expected_distances"], np.float32), rtol=1e-6)
    assert pred.tolist() == g["expected_predecessors"]

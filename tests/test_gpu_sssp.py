"""SSSP parity: fp32/fp64 distances bit-identical to the oracle's min-plus fixed
point; predecessors = smallest tight in-neighbour (golden vectors agree)."""
import numpy as np
import pytest

from conftest import dataset_path
from gpu_util import host, make_graph, plc
from oracle import graph as og
from oracle import rmat
from oracle import sssp as osssp

pytestmark = pytest.mark.gpu


def run(h, G, source, cutoff=1e38, pred=True):
    v, d, p = plc().sssp(h, G, source, cutoff, pred, False)
    return host(v), host(d), host(p)


def test_c_golden(golden):
    g = golden["sssp_c"]
    for transposed in (False, True):
        h, G = make_graph(g["src"], g["dst"], g["w"], transposed=transposed, renumber=False)
        v, dist, pred = run(h, G, g["source"], g["cutoff"])
        exp = np.asarray(g["expected_distances"], np.float32)
        assert np.allclose(dist, exp[v], rtol=1e-6)
        assert np.array_equal(pred, np.asarray(g["expected_predecessors"])[v])


def test_c_golden_double(golden):
    g = golden["sssp_c"]
    h, G = make_graph(g["src"], g["dst"], g["w"], transposed=True, renumber=False, wdtype=np.float64)
    v, dist, pred = run(h, G, g["source"], g["cutoff"])
    exp = np.asarray(g["expected_distances"], np.float64)
    exp[2] = np.finfo(np.float64).max
    assert np.allclose(dist, exp[v], rtol=1e-12)
    assert np.array_equal(pred, np.asarray(g["expected_predecessors"])[v])


@pytest.mark.parametrize("name", ["karate.csv", "dolphins.csv", "Simple_1", "Simple_2"])
def test_pylib_golden(golden, name):
    p = golden["sssp_pylib"]
    exp = p[name]
    if "src" in exp:
        s, d, w = exp["src"], exp["dst"], np.asarray(exp["w"], np.float32)
    else:
        s, d, w = og.read_csv(dataset_path(name))
    h, G = make_graph(s, d, w, renumber=False)
    v, dist, pred = run(h, G, exp["source"], p["cutoff"])
    assert np.array_equal(dist, np.asarray(exp["distance"], np.float32)[v])
    G2 = og.create_graph(s, d, np.asarray(w, np.float32), renumber=False)
    rd, rp = osssp.sssp(G2.num_vertices, G2.offsets, G2.indices, G2.weights, exp["source"], p["cutoff"])
    assert np.array_equal(pred, rp[v])


@pytest.mark.parametrize("scale,symmetric", [(10, True), (13, True), (12, False)])
def test_rmat_weighted(scale, symmetric):
    s, d = rmat.rmat(scale, 16 << scale)
    w = rmat.rmat_weights(s.size, seed=43).astype(np.float64)
    s, d, w = og.symmetrize_dedup(s, d, w, symmetrize=symmetric)
    h, G = make_graph(s, d, w, renumber=True, symmetric=symmetric)
    src = int(s[0])
    v, dist, pred = run(h, G, src)
    n_ext = int(max(s.max(), d.max())) + 1
    G2 = og.create_graph(s, d, w.astype(np.float32), renumber=False, vertices=np.arange(n_ext))
    key = np.empty(n_ext, np.int64)
    key[v] = np.arange(v.size)
    absent = np.setdiff1d(np.arange(n_ext), v)
    key[absent] = v.size + np.arange(absent.size)
    rd, rp = osssp.sssp(n_ext, G2.offsets, G2.indices, G2.weights, src, tie_key=key)
    assert np.array_equal(dist, rd[v])
    assert np.array_equal(pred, rp[v])


def test_cutoff():
    s, d = rmat.rmat(11, 16 << 11)
    w = rmat.rmat_weights(s.size).astype(np.float64)
    s, d, w = og.symmetrize_dedup(s, d, w)
    h, G = make_graph(s, d, w, renumber=True, symmetric=True)
    src = int(s[0])
    v, dist, pred = run(h, G, src, cutoff=0.05)
    G2 = og.create_graph(s, d, w.astype(np.float32), renumber=False,
                         vertices=np.arange(int(max(s.max(), d.max())) + 1))
    rd, _ = osssp.sssp(G2.num_vertices, G2.offsets, G2.indices, G2.weights, src, cutoff=0.05)
    assert np.array_equal(dist, rd[v])


def test_unweighted_rejected():
    h, G = make_graph([0, 1], [1, 2], None, renumber=False)
    with pytest.raises(ValueError, match="unweighted"):
        run(h, G, 0)


def test_bad_source():
    h, G = make_graph([0, 1], [1, 2], [1.0, 1.0], renumber=False)
    with pytest.raises(ValueError):
        run(h, G, 9)


@pytest.mark.parametrize("scale,wdtype", [(20, np.float32), (18, np.float64)])
def test_rmat_uniform_weights_vs_compiled_oracle(scale, wdtype):
    """The reference's SSSP test size (RMAT(20, ...), sssp_test.cpp:305), symmetric
    with the bench's uniform [0, 1) weights (cugraph_funcs.py:56-58), from 4 sources
    (the largest hub, two random vertices, a low-degree vertex): distances bit-exact
    against the compiled near-far restatement (oracle/cpu_sssp.c) on the library's own
    CSR, and every predecessor the smallest tight in-neighbour."""
    import torch
    from oracle import cpu_native
    p = plc()
    h = p.ResourceHandle()
    n = 16 << scale
    s, d = p.generators.generate_rmat_edgelist(h, scale, n, 0.57, 0.19, 0.19, 42, False, True)
    w = p.generators.generate_edge_weights(h, n, 43)
    if wdtype == np.float64:
        w = w.to(torch.float64)
    s, d, w = p.generators.symmetrize_dedup(h, s, d, w, True)
    G = p.SGGraph(h, p.GraphProperties(is_symmetric=True, is_multigraph=False), s, d, w, store_transposed=False,
                  renumber=True)
    off, idx, ww = G.adjacency(h, transposed=False)
    off, idx, ww = host(off).astype(np.int64), host(idx), host(ww)
    assert ww.dtype == wdtype
    V = off.size - 1
    rng = np.random.default_rng(5)
    nm = None
    for k in range(4):
        if nm is None:  # the first call (from an edge's source) also gives the number map
            ext = int(s[0])
        else:
            ext = int(nm[[0, int(rng.integers(V)), V - 1][k - 1]])  # the largest hub, a random, the last vertex
        v, dist, pred = run(h, G, ext)
        nm = v if nm is None else nm
        assert np.array_equal(v, nm)
        src_int = int(np.nonzero(nm == ext)[0][0])
        t, rd, rp, rounds = cpu_native.sssp(off, idx, ww, src_int)
        assert np.array_equal(dist, rd), f"source {src_int}: distances differ from the compiled oracle"
        want = np.where(rp >= 0, nm[np.maximum(rp, 0)], -1)
        assert np.array_equal(pred.astype(np.int64), want.astype(np.int64)), f"source {src_int}: predecessors"
        reached = int((rd < np.finfo(wdtype).max).sum())
        print(f"RMAT-{scale} {np.dtype(wdtype).name} SSSP from internal {src_int}: reached {reached} of {V}, "
              f"GPU rounds {h.last_iterations()}, oracle rounds {rounds} ({t:.2f} s)")

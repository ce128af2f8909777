"""Katz / eigenvector centrality / HITS (csrc/centrality.hip) through the C ABI:
the reference's C-test golden vectors, the oracle (oracle/centrality.py) on RMAT
graphs, and the cugraph wrappers against NetworkX."""
import numpy as np
import pytest

from conftest import dataset_path
from gpu_util import host, make_graph, plc
from oracle import centrality as oc
from oracle import graph as og
from oracle import rmat

pytestmark = pytest.mark.gpu


def near(a, b, eps):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= np.maximum(eps * np.maximum(np.abs(a), np.abs(b)), 1e-6))


def by_vertex(v, x):
    out = np.zeros(int(host(v).max()) + 1)
    out[host(v)] = host(x)
    return out


@pytest.mark.parametrize("transposed", [True, False])
def test_katz_c_golden(golden, transposed):
    g = golden["katz_c"]
    h, G = make_graph(g["src"], g["dst"], g["w"], transposed=transposed, renumber=False)
    v, x = plc().katz_centrality(h, G, None, g["alpha"], g["beta"], g["epsilon"], g["max_iterations"], False)
    assert near(by_vertex(v, x), g["expected"], g["tol"])


def test_eigenvector_c_golden(golden):
    g = golden["eigenvector_c"]
    h, G = make_graph(g["src"], g["dst"], g["w"], transposed=True, renumber=False)
    v, x = plc().eigenvector_centrality(h, G, g["epsilon"], g["max_iterations"], False)
    assert near(by_vertex(v, x), g["expected"], g["tol"])


@pytest.mark.parametrize("transposed", [True, False])
def test_hits_c_golden(golden, transposed):
    import torch
    for c in golden["hits_c"]["cases"]:
        h, G = make_graph(c["src"], c["dst"], np.ones(len(c["src"])), transposed=transposed, renumber=False)
        gv = gx = None
        if "initial_vertices" in c:
            gv = torch.tensor(c["initial_vertices"], dtype=torch.int32, device="cuda")
            gx = torch.tensor(c["initial_hubs"], dtype=torch.float32, device="cuda")
        v, hb, au = plc().hits(h, G, c["epsilon"], c["max_iterations"], gv, gx, False, False)
        n = c["num_vertices"]
        hubs = np.zeros(n)
        auth = np.zeros(n)
        hubs[host(v)] = host(hb)
        auth[host(v)] = host(au)
        assert near(hubs, c["hubs"], golden["hits_c"]["tol"]), c["name"]
        assert near(auth, c["authorities"], golden["hits_c"]["tol"]), c["name"]


def rmat_graph(scale, weighted, seed=9):
    s, d = rmat.rmat(scale, 16 << scale, seed=seed)
    w = rmat.rmat_weights(s.size, seed=seed + 1).astype(np.float64) if weighted else None
    return og.symmetrize_dedup(s, d, w)


@pytest.mark.parametrize("weighted", [False, True])
def test_rmat_vs_oracle(weighted):
    s, d, w = rmat_graph(11, weighted)
    w32 = None if w is None else w.astype(np.float32)
    ww = None if w32 is None else w32.astype(np.float64)
    h, G = make_graph(s, d, w32, transposed=True, renumber=True, symmetric=True)
    og_g = og.create_graph(s, d, ww, store_transposed=True, renumber=True)
    cs, cd, cw = og_g.coo()  # (minor, major) pairs of the CSC: source, destination
    nv = og_g.num_vertices
    ext = og_g.number_map

    def ext_of(v, x):
        out = np.zeros(int(ext.max()) + 1)
        out[host(v)] = host(x)
        return out[ext]

    degmax = np.bincount(s).max()
    alpha = 1.0 / (degmax + 1.0)
    v, x = plc().katz_centrality(h, G, None, alpha, 1.0, 1e-8, 1000, False)
    ref = oc.katz(nv, cs, cd, cw, alpha, 1.0, 1e-8, 1000)
    assert np.max(np.abs(ext_of(v, x) - ref)) < 1e-5
    v, x = plc().eigenvector_centrality(h, G, 1e-7, 1000, False)
    ref = oc.eigenvector_centrality(nv, cs, cd, cw, 1e-7, 1000)
    assert np.max(np.abs(ext_of(v, x) - ref)) < 1e-4
    v, hb, au = plc().hits(h, G, 1e-6, 100, None, None, True, False)
    rh, ra, _, _ = oc.hits(nv, cs, cd, 1e-6, 100)
    assert np.max(np.abs(ext_of(v, hb) - rh)) < 1e-5 and np.max(np.abs(ext_of(v, au) - ra)) < 1e-5


def test_katz_not_converged():
    h, G = make_graph([0, 1, 2], [1, 2, 0], None, transposed=True, renumber=False)
    with pytest.raises(RuntimeError, match="failed to converge"):
        plc().katz_centrality(h, G, None, 0.5, 1.0, 1e-12, 2, False)


def test_cugraph_wrappers_vs_networkx():
    nx = pytest.importorskip("networkx")
    import cugraph
    import pandas as pd
    a = np.loadtxt(dataset_path("karate.csv"), ndmin=2)
    df = pd.DataFrame({"0": a[:, 0].astype(np.int32), "1": a[:, 1].astype(np.int32)})
    G = cugraph.Graph()
    G.from_cudf_edgelist(df, "0", "1", store_transposed=True)
    Gx = nx.Graph()
    Gx.add_edges_from(zip(df["0"].tolist(), df["1"].tolist()))
    k = cugraph.katz_centrality(G, alpha=0.05, max_iter=1000, tol=1e-10)
    ref = nx.katz_centrality(Gx, alpha=0.05, beta=1.0, max_iter=1000, tol=1e-12, normalized=True)
    got = dict(zip(k["vertex"].tolist(), k["katz_centrality"].tolist()))
    assert max(abs(got[n] - ref[n]) for n in ref) < 1e-5
    hres = cugraph.hits(G, max_iter=1000, tol=1e-10)
    rh, ra = nx.hits(Gx, max_iter=1000, tol=1e-12)
    gh = dict(zip(hres["vertex"].tolist(), hres["hubs"].tolist()))
    ga = dict(zip(hres["vertex"].tolist(), hres["authorities"].tolist()))
    assert max(abs(gh[n] - rh[n]) for n in rh) < 1e-5 and max(abs(ga[n] - ra[n]) for n in ra) < 1e-5
    e = cugraph.eigenvector_centrality(G, max_iter=1000, tol=1e-6)
    ref = nx.eigenvector_centrality_numpy(Gx)
    ge = dict(zip(e["vertex"].tolist(), e["eigenvector_centrality"].tolist()))
    assert max(abs(ge[n] - ref[n]) for n in ref) < 1e-3
    kd = cugraph.katz_centrality(Gx, alpha=0.05, max_iter=1000, tol=1e-10)
    assert set(kd) == set(Gx.nodes())

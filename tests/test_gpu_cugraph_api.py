"""cugraph Python surface (cugraph-forked_amd/cugraph) following the reference's
python/cugraph/cugraph/tests: NetworkX is the oracle there (test_pagerank.py:99-131,
204-219; test_bfs.py:191-257; test_louvain.py:96-103), plus the pylibcugraph golden
vectors for karate."""
import numpy as np
import pandas as pd
import pytest

from conftest import dataset_path

pytestmark = pytest.mark.gpu

nx = pytest.importorskip("networkx")


def cg():
    import cugraph
    return cugraph


def read_df(name):
    a = np.loadtxt(dataset_path(name), ndmin=2)
    return pd.DataFrame({"0": a[:, 0].astype(np.int32), "1": a[:, 1].astype(np.int32),
                         "2": a[:, 2].astype(np.float32)})


def nx_graph(name, directed=False):
    df = read_df(name)
    G = nx.DiGraph() if directed else nx.Graph()
    G.add_weighted_edges_from(zip(df["0"].tolist(), df["1"].tolist(), df["2"].astype(float).tolist()))
    return G


@pytest.mark.parametrize("name", ["karate.csv", "dolphins.csv", "netscience.csv"])
@pytest.mark.parametrize("directed", [False, True])
def test_pagerank_vs_networkx(name, directed):
    df = read_df(name)
    G = cg().DiGraph() if directed else cg().Graph()
    G.from_cudf_edgelist(df, source="0", destination="1", store_transposed=True)
    max_iter, tol = 100, 1e-5
    pr = cg().pagerank(G, alpha=0.85, max_iter=max_iter, tol=tol)
    assert list(pr.columns) == ["vertex", "pagerank"]
    # test_pagerank.py: nx.pagerank(max_iter*2, tol*0.01), < 1% of vertices off by more than 1.1*tol
    ref = nx.pagerank(nx_graph(name, directed), alpha=0.85, max_iter=max_iter * 2, tol=tol * 0.01, weight=None)
    got = dict(zip(pr["vertex"].tolist(), pr["pagerank"].tolist()))
    assert set(got) == set(ref)
    bad = sum(abs(got[v] - ref[v]) > 1.1 * tol for v in ref)
    assert bad < 0.01 * len(ref)


def test_pagerank_karate_golden(golden):
    exp = np.asarray(golden["pagerank_pylib"]["karate.csv"])
    df = read_df("karate.csv")
    G = cg().DiGraph()
    G.from_cudf_edgelist(df, source="0", destination="1", renumber=False, store_transposed=True)
    pr = cg().pagerank(G, alpha=0.85, max_iter=500, tol=1e-6)
    got = pr.sort_values("vertex")["pagerank"].to_numpy()
    assert np.allclose(got, exp, rtol=1e-4)
    assert abs(pr["pagerank"].sum() - 1.0) < 1e-5


def test_pagerank_networkx_input_and_personalization():
    Gx = nx_graph("karate.csv")
    pr = cg().pagerank(Gx, max_iter=500, tol=1e-8)
    ref = nx.pagerank(Gx, max_iter=1000, tol=1e-12)
    assert set(pr) == set(ref)
    assert max(abs(pr[v] - ref[v]) for v in ref) < 1e-5
    pers = pd.DataFrame({"vertex": [1, 2], "values": [0.3, 0.7]})
    df = read_df("karate.csv")
    G = cg().Graph()
    G.from_cudf_edgelist(df, source="0", destination="1", store_transposed=True)
    ppr = cg().pagerank(G, personalization=pers, max_iter=500, tol=1e-8)
    ref = nx.pagerank(nx_graph("karate.csv"), personalization={1: 0.3, 2: 0.7}, max_iter=1000, tol=1e-12,
                      weight=None)
    got = dict(zip(ppr["vertex"].tolist(), ppr["pagerank"].tolist()))
    assert max(abs(got[v] - ref[v]) for v in ref) < 1e-5


@pytest.mark.parametrize("name", ["karate.csv", "dolphins.csv", "netscience.csv", "polbooks.csv"])
def test_bfs_vs_networkx(name):
    df = read_df(name)
    G = cg().Graph()
    G.from_cudf_edgelist(df, source="0", destination="1")
    start = int(df["0"].iloc[0])
    res = cg().bfs(G, start)
    assert list(res.columns) == ["vertex", "distance", "predecessor"]
    Gx = nx_graph(name)
    ref = nx.single_source_shortest_path_length(Gx, start)
    d = dict(zip(res["vertex"].tolist(), res["distance"].tolist()))
    p = dict(zip(res["vertex"].tolist(), res["predecessor"].tolist()))
    for v, dist in d.items():
        if v in ref:
            assert dist == ref[v]
            if v != start:
                assert ref[p[v]] + 1 == dist and Gx.has_edge(p[v], v)
        else:
            assert dist == 2**31 - 1 and p[v] == -1
    # depth limit
    lim = cg().bfs(G, start, depth_limit=1)
    assert lim["distance"][lim["distance"] < 2**31 - 1].max() <= 1


def test_bfs_argument_errors():
    df = read_df("karate.csv")
    G = cg().Graph()
    G.from_cudf_edgelist(df, source="0", destination="1")
    with pytest.raises(TypeError):
        cg().bfs(G, 1, i_start=1)
    with pytest.raises(TypeError):
        cg().bfs(G)
    with pytest.raises(ValueError):
        cg().bfs(G, 1000)


@pytest.mark.parametrize("name", ["karate.csv", "dolphins.csv"])
def test_sssp_vs_networkx(name):
    df = read_df(name)
    df["2"] = (np.arange(len(df)) % 7 + 1).astype(np.float32)  # non-trivial weights
    G = cg().Graph()
    G.from_cudf_edgelist(df, source="0", destination="1", edge_attr="2")
    src = int(df["0"].iloc[0])
    res = cg().sssp(G, src)
    assert list(res.columns) == ["distance", "vertex", "predecessor"]
    Gx = nx.Graph()
    for a, b, w in zip(df["0"], df["1"], df["2"]):  # min weight on duplicates, as cugraph.Graph
        w = float(w)
        if not Gx.has_edge(a, b) or Gx[a][b]["weight"] > w:
            Gx.add_edge(int(a), int(b), weight=w)
    ref = nx.single_source_dijkstra_path_length(Gx, src)
    got = dict(zip(res["vertex"].tolist(), res["distance"].tolist()))
    for v, dv in ref.items():
        assert abs(got[v] - dv) < 1e-4
    assert cg().shortest_path_length(G, src, int(df["1"].iloc[3])) == pytest.approx(ref[int(df["1"].iloc[3])])


@pytest.mark.parametrize("name", ["karate.csv", "dolphins.csv", "netscience.csv"])
def test_louvain_vs_networkx(name):
    df = read_df(name)
    G = cg().Graph()
    G.from_cudf_edgelist(df, source="0", destination="1", edge_attr="2")
    parts, q = cg().louvain(G)
    assert list(parts.columns) == ["vertex", "partition"]
    Gx = nx_graph(name)
    comm = {}
    for v, c in zip(parts["vertex"].tolist(), parts["partition"].tolist()):
        comm.setdefault(c, set()).add(v)
    qx = nx.community.modularity(Gx, list(comm.values()))
    assert abs(q - qx) < 1e-4  # test_louvain.py:96-103
    ref_q = nx.community.modularity(Gx, nx.community.louvain_communities(Gx, seed=42))
    assert q > 0.82 * ref_q


def test_louvain_directed_and_networkx_input():
    df = read_df("karate.csv")
    G = cg().DiGraph()
    G.from_cudf_edgelist(df, source="0", destination="1", edge_attr="2")
    with pytest.raises(ValueError):
        cg().louvain(G)
    parts, q = cg().louvain(nx_graph("karate.csv"))
    assert set(parts) == set(nx_graph("karate.csv").nodes()) and q > 0.35


def test_graph_queries():
    df = read_df("karate.csv")
    G = cg().Graph()
    G.from_cudf_edgelist(df, source="0", destination="1", edge_attr="2")
    assert not G.is_directed() and G.is_weighted()
    assert G.number_of_vertices() == 34 and G.number_of_edges() == 78
    el = G.view_edge_list()
    assert len(el) == 78 and set(el.columns) == {"src", "dst", "weights"}
    with pytest.raises(RuntimeError):
        G.from_cudf_edgelist(df, source="0", destination="1")
    with pytest.raises(ValueError):
        cg().Graph().from_cudf_edgelist(df, source="x", destination="1")

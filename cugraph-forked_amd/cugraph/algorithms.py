"""cugraph algorithm wrappers (reference link_analysis/pagerank.py:61-244,
traversal/bfs.py:127-262, traversal/sssp.py:132-260, community/louvain.py:23-101).

Same names, argument order, defaults, result columns and error types; the
inputs may also be NetworkX graphs (results then use the NetworkX node labels, as
the reference's ``ensure_cugraph_obj_for_nx`` / ``df_score_to_dictionary``)."""
from __future__ import annotations

import warnings

import numpy as np

from .structure import DiGraph, Graph


def _plc():
    import pylibcugraph
    return pylibcugraph


def _is_nx(G):
    try:
        import networkx as nx
    except ImportError:
        return False
    return isinstance(G, nx.Graph)


class _NxView:
    """A NetworkX graph as a cugraph Graph over integer labels 0..n-1."""

    def __init__(self, nxG, weight="weight", store_transposed=False):
        import pandas as pd
        self.nodes = list(nxG.nodes())
        index = {n: i for i, n in enumerate(self.nodes)}
        rows = [(index[u], index[v], float(d.get(weight, 1.0)) if weight else 1.0)
                for u, v, d in nxG.edges(data=True)]
        arr = np.array(rows, dtype=np.float64).reshape(-1, 3)
        df = pd.DataFrame({"src": arr[:, 0].astype(np.int64), "dst": arr[:, 1].astype(np.int64), "w": arr[:, 2]})
        weighted = any("weight" in d for _, _, d in nxG.edges(data=True)) and weight is not None
        self.G = DiGraph() if nxG.is_directed() else Graph()
        self.G.from_pandas_edgelist(df, "src", "dst", "w" if weighted else None, renumber=True,
                                    store_transposed=store_transposed)
        self.index = index

    def label(self, ids):
        return [self.nodes[int(i)] if int(i) >= 0 else -1 for i in ids]

    def ids(self, labels):
        if np.isscalar(labels) or not hasattr(labels, "__len__"):
            labels = [labels]
        try:
            return [self.index[x] for x in labels]
        except KeyError:
            raise ValueError("A provided vertex was not valid") from None


def _frame_col(df, name):
    import torch
    c = df[name]
    if isinstance(c, torch.Tensor):
        return c
    if hasattr(c, "to_numpy"):
        c = c.to_numpy()
    return torch.as_tensor(np.asarray(c))


def _cuda_like(t, dtype):
    return t.to(dtype).cuda()


def _vertex_dtype(G):
    return G.edgelist["src"].dtype


def pagerank(G, alpha=0.85, personalization=None, precomputed_vertex_out_weight=None, max_iter=100, tol=1.0e-5,
             nstart=None, weight=None, dangling=None):
    """link_analysis/pagerank.py:61-244.  Returns DataFrame ['vertex', 'pagerank']
    (dict {node: score} for a NetworkX input)."""
    import pandas as pd
    import torch
    nxv = None
    if _is_nx(G):
        nxv = _NxView(G, weight or "weight", store_transposed=True)
        G = nxv.G
    if G.store_transposed is False:
        warnings.warn("Pagerank expects the 'store_transposed' flag to be set to 'True' for optimal performance "
                      "during the graph creation", UserWarning)
    p = _plc()
    vt = _vertex_dtype(G)
    wt = torch.float32 if G.edgelist["weights"] is None else G.edgelist["weights"].dtype

    def pair(df, vcol, xcol):
        if df is None:
            return None, None
        if nxv is not None:
            v = torch.as_tensor(nxv.ids(list(df[vcol])), dtype=torch.int64)
        else:
            v = _frame_col(df, vcol)
        return _cuda_like(v, vt), _cuda_like(_frame_col(df, xcol), wt)

    gv, gx = pair(nstart, "vertex", "values")
    ov, ox = pair(precomputed_vertex_out_weight, "vertex", "sums")
    h = p.ResourceHandle()
    if personalization is not None:
        pv, px = pair(personalization, "vertex", "values")
        vertex, values = p.personalized_pagerank(h, G._plc_graph, ov, ox, gv, gx, pv, px, alpha, tol, max_iter, False)
    else:
        vertex, values = p.pagerank(h, G._plc_graph, ov, ox, gv, gx, alpha, tol, max_iter, False)
    df = pd.DataFrame({"vertex": vertex.cpu().numpy(), "pagerank": values.cpu().numpy()})
    if nxv is not None:
        return dict(zip(nxv.label(df["vertex"]), df["pagerank"]))
    return df


def _starts(G, start, i_start, directed, nxv):
    if start is not None and i_start is not None:
        raise TypeError("cannot specify both 'start' and 'i_start'")
    if start is None and i_start is None:
        raise TypeError("must specify 'start' or 'i_start', but not both")
    if directed is not None:
        raise TypeError("'directed' cannot be specified for a Graph-type input")
    start = start if start is not None else i_start
    if nxv is not None:
        return nxv.ids(start)
    if hasattr(start, "columns"):
        start = start[start.columns[0]]
    if hasattr(start, "to_numpy"):
        start = start.to_numpy()
    s = np.atleast_1d(np.asarray(start)).astype(np.int64)
    for x in s:
        if not G.has_node(int(x)):
            raise ValueError("A provided vertex was not valid")
    return s.tolist()


def bfs(G, start=None, depth_limit=None, i_start=None, directed=None, return_predecessors=True):
    """traversal/bfs.py:127-262.  Returns DataFrame ['vertex', 'distance', 'predecessor']."""
    import pandas as pd
    import torch
    nxv = None
    if _is_nx(G):
        nxv = _NxView(G)
        G = nxv.G
    starts = _starts(G, start, i_start, directed, nxv)
    p = _plc()
    src = torch.as_tensor(starts, dtype=_vertex_dtype(G)).cuda()
    dist, pred, vertex = p.bfs(p.ResourceHandle(), G._plc_graph, src, False,
                               depth_limit if depth_limit is not None else -1, return_predecessors, False)
    df = pd.DataFrame({"vertex": vertex.cpu().numpy(), "distance": dist.cpu().numpy(),
                       "predecessor": (pred.cpu().numpy() if return_predecessors
                                       else np.full(vertex.numel(), -1, dtype=vertex.cpu().numpy().dtype))})
    if nxv is not None:
        df["vertex"] = nxv.label(df["vertex"])
        df["predecessor"] = nxv.label(df["predecessor"])
    return df


def sssp(G, source=None, method=None, directed=None, return_predecessors=None, unweighted=None, overwrite=None,
         indices=None, cutoff=None, edge_attr="weight"):
    """traversal/sssp.py:132-260.  Returns DataFrame ['distance', 'vertex', 'predecessor'];
    unweighted graphs use weight 1.0 (simpleGraph.py:840-843)."""
    import pandas as pd
    if source is None and indices is None:
        raise TypeError("must specify 'source' or 'indices', but not both")
    if source is not None and indices is not None:
        raise TypeError("must specify 'source' or 'indices', but not both")
    source = source if source is not None else indices
    nxv = None
    if _is_nx(G):
        nxv = _NxView(G, edge_attr)
        G = nxv.G
        source = nxv.ids(source)[0]
    elif not G.has_node(int(source)):
        raise ValueError("Starting vertex should be between 0 to number of vertices")
    if cutoff is None:
        cutoff = np.inf
    p = _plc()
    vertex, dist, pred = p.sssp(p.ResourceHandle(), G._weighted_plc_graph(), int(source), float(cutoff), True, False)
    df = pd.DataFrame({"distance": dist.cpu().numpy(), "vertex": vertex.cpu().numpy(),
                       "predecessor": pred.cpu().numpy()})
    if nxv is not None:
        df["vertex"] = nxv.label(df["vertex"])
        df["predecessor"] = nxv.label(df["predecessor"])
    return df


def shortest_path(G, source=None, method=None, directed=None, return_predecessors=None, unweighted=None,
                  overwrite=None, indices=None):
    """Alias of sssp (traversal/sssp.py)."""
    return sssp(G, source, method, directed, return_predecessors, unweighted, overwrite, indices)


def shortest_path_length(G, source, target=None):
    """traversal/sssp.py shortest_path_length: DataFrame ['vertex', 'distance'] or one distance."""
    df = sssp(G, source)
    if target is not None:
        hit = df.loc[df["vertex"] == target]
        if hit.empty:
            raise ValueError("Graph does not contain target vertex")
        return hit.iloc[0]["distance"]
    return df[["vertex", "distance"]].reset_index(drop=True)


def louvain(G, max_iter=100, resolution=1.0):
    """community/louvain.py:23-101.  Returns (DataFrame ['vertex', 'partition'], modularity)."""
    import pandas as pd
    nxv = None
    if _is_nx(G):
        nxv = _NxView(G)
        G = nxv.G
    if G.is_directed():
        raise ValueError("input graph must be undirected")
    p = _plc()
    vertex, part, q = p.louvain(p.ResourceHandle(), G._weighted_plc_graph(), max_iter, resolution, False)
    df = pd.DataFrame({"vertex": vertex.cpu().numpy(), "partition": part.cpu().numpy()})
    if nxv is not None:
        return dict(zip(nxv.label(df["vertex"]), df["partition"])), q
    return df, q


def _max_degree(G):
    import torch
    e = G.edgelist
    ids = torch.cat([e["src"], e["dst"]]) if G.is_directed() else e["src"]
    return int(torch.bincount(ids.to(torch.int64)).max().item()) if ids.numel() else 0


def katz_centrality(G, alpha=None, beta=1.0, max_iter=100, tol=1.0e-6, nstart=None, normalized=True):
    """centrality/katz_centrality.py:24-170.  Returns DataFrame ['vertex', 'katz_centrality']
    (dict for a NetworkX input).  As the reference, ``nstart`` is passed as the betas."""
    import pandas as pd
    import torch
    nxv = None
    if _is_nx(G):
        nxv = _NxView(G, store_transposed=True)
        G = nxv.G
    if alpha is None:
        alpha = 1.0 / _max_degree(G)
    if alpha <= 0.0:
        raise ValueError(f"'alpha' must be a positive float or None, got: {alpha}")
    if not isinstance(beta, float) or beta <= 0.0:
        raise ValueError(f"'beta' must be a positive float or None, got: {beta}")
    if not isinstance(max_iter, int) or max_iter <= 0:
        raise ValueError(f"'max_iter' must be a positive integer, got: {max_iter}")
    if not isinstance(tol, float) or tol <= 0.0:
        raise ValueError(f"'tol' must be a positive float, got: {tol}")
    betas = None
    if nstart is not None:
        wt = torch.float32 if G.edgelist["weights"] is None else G.edgelist["weights"].dtype
        betas = _cuda_like(_frame_col(nstart, "values"), wt)
    p = _plc()
    vertex, values = p.katz_centrality(p.ResourceHandle(), G._plc_graph, betas, alpha, beta, tol, max_iter, False)
    df = pd.DataFrame({"vertex": vertex.cpu().numpy(), "katz_centrality": values.cpu().numpy()})
    if nxv is not None:
        return dict(zip(nxv.label(df["vertex"]), df["katz_centrality"]))
    return df


def eigenvector_centrality(G, max_iter=100, tol=1.0e-6):
    """centrality/eigenvector_centrality.py.  Returns DataFrame ['vertex', 'eigenvector_centrality']."""
    import pandas as pd
    nxv = None
    if _is_nx(G):
        nxv = _NxView(G, store_transposed=True)
        G = nxv.G
    p = _plc()
    vertex, values = p.eigenvector_centrality(p.ResourceHandle(), G._plc_graph, tol, max_iter, False)
    df = pd.DataFrame({"vertex": vertex.cpu().numpy(), "eigenvector_centrality": values.cpu().numpy()})
    if nxv is not None:
        return dict(zip(nxv.label(df["vertex"]), df["eigenvector_centrality"]))
    return df


def hits(G, max_iter=100, tol=1.0e-5, nstart=None, normalized=True):
    """link_analysis/hits.py:26-120.  Returns DataFrame ['vertex', 'hubs', 'authorities']
    ((hubs dict, authorities dict) for a NetworkX input)."""
    import pandas as pd
    import torch
    nxv = None
    if _is_nx(G):
        nxv = _NxView(G, store_transposed=True)
        G = nxv.G
    if G.store_transposed is False:
        warnings.warn("HITS expects the 'store_transposed' flag to be set to 'True' for optimal performance during "
                      "the graph creation", UserWarning)
    gv = gx = None
    if nstart is not None:
        wt = torch.float32 if G.edgelist["weights"] is None else G.edgelist["weights"].dtype
        v = (torch.as_tensor(nxv.ids(list(nstart["vertex"]))) if nxv is not None else _frame_col(nstart, "vertex"))
        gv, gx = _cuda_like(v, _vertex_dtype(G)), _cuda_like(_frame_col(nstart, "values"), wt)
    p = _plc()
    vertex, hubs_, auth = p.hits(p.ResourceHandle(), G._plc_graph, tol, max_iter, gv, gx, normalized, False)
    df = pd.DataFrame({"vertex": vertex.cpu().numpy(), "hubs": hubs_.cpu().numpy(),
                       "authorities": auth.cpu().numpy()})
    if nxv is not None:
        lab = nxv.label(df["vertex"])
        return dict(zip(lab, df["hubs"])), dict(zip(lab, df["authorities"]))
    return df

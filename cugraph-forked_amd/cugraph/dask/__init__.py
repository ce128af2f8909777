"""Multi-GPU algorithms, one process per GPU (reference ``python/cugraph/cugraph/dask``:
``link_analysis/pagerank.py``, ``traversal/bfs.py``, ``traversal/sssp.py``,
``community/louvain.py``).

The reference runs on a dask-cuda cluster: the caller holds a dask_cudf edge
list, the algorithms return a dask_cudf DataFrame whose partitions live on the
workers.  Here the workers ARE the processes (``torch.distributed.run``): every
rank calls each function collectively with the same arguments, the graph is a
``cugraph.Graph`` built by ``from_dask_cudf_edgelist`` from the rank's own
partition, and the result is the rank's partition of the reference's dask frame
(a pandas DataFrame of the vertices this rank owns, external ids); ``gather``
concatenates the partitions on every rank.  Setup:
``cugraph.dask.comms.comms.initialize()`` / ``destroy()``.
"""
from __future__ import annotations

import numpy as np

from .comms import comms as _comms


def _plc():
    import pylibcugraph
    return pylibcugraph


def _check(G):
    if not getattr(G, "is_distributed", lambda: False)():
        raise TypeError("cugraph.dask algorithms need a graph built with Graph.from_dask_cudf_edgelist")


def _pairs(df, vcol, xcol, vt, wt):
    """(vertex, value) columns of this rank's partition of a DataFrame -> CUDA tensors."""
    import torch
    if df is None:
        return None, None
    v = df[vcol].to_numpy() if hasattr(df[vcol], "to_numpy") else np.asarray(df[vcol])
    x = df[xcol].to_numpy() if hasattr(df[xcol], "to_numpy") else np.asarray(df[xcol])
    return (torch.as_tensor(np.ascontiguousarray(v)).to(vt).cuda(),
            torch.as_tensor(np.ascontiguousarray(x)).to(wt).cuda())


def pagerank(input_graph, alpha=0.85, personalization=None, precomputed_vertex_out_weight=None, max_iter=100,
             tol=1.0e-5, nstart=None):
    """dask/link_analysis/pagerank.py:129-337.  personalization / nstart /
    precomputed_vertex_out_weight: this rank's partition of the (vertex, values |
    sums) frame.  Returns this rank's rows of DataFrame ['vertex', 'pagerank']."""
    import pandas as pd
    import torch
    _check(input_graph)
    p = _plc()
    h = _comms.get_default_handle()
    G = input_graph
    vt = G.edgelist["src"].dtype
    wt = torch.float32 if G.edgelist["weights"] is None else G.edgelist["weights"].dtype
    gv, gx = _pairs(nstart, "vertex", "values", vt, wt)
    ov, ox = _pairs(precomputed_vertex_out_weight, "vertex", "sums", vt, wt)
    if personalization is not None:
        pv, px = _pairs(personalization, "vertex", "values", vt, wt)
        vertex, values = p.personalized_pagerank(h, G._plc_graph, ov, ox, gv, gx, pv, px, alpha, tol, max_iter,
                                                 False)
    else:
        vertex, values = p.pagerank(h, G._plc_graph, ov, ox, gv, gx, alpha, tol, max_iter, False)
    return pd.DataFrame({"vertex": vertex.cpu().numpy(), "pagerank": values.cpu().numpy()})


def bfs(input_graph, start, depth_limit=None, return_distances=True, check_start=True):
    """dask/traversal/bfs.py:56-203.  ``start``: a vertex id or a list of them (the
    same on every rank).  Returns this rank's rows of ['vertex', 'distance',
    'predecessor'] (predecessor -1 when none)."""
    import pandas as pd
    import torch
    import torch.distributed as dist
    _check(input_graph)
    p = _plc()
    h = _comms.get_default_handle()
    G = input_graph
    starts = np.atleast_1d(np.asarray(start)).astype(np.int64)
    if check_start:
        e = G.edgelist
        present = torch.zeros(starts.size, dtype=torch.int64, device=_comms.collective_device())
        for i, x in enumerate(starts.tolist()):
            present[i] = int(((e["src"] == x).any() | (e["dst"] == x).any()).item())
        dist.all_reduce(present, op=dist.ReduceOp.MAX)
        if not bool((present > 0).all()):
            raise ValueError("start vertex is not present in the graph")
    mine = starts if dist.get_rank() == 0 else starts[:0]
    src = torch.as_tensor(mine).to(G.edgelist["src"].dtype).cuda()
    d, pred, vertex = p.bfs(h, G._plc_graph, src, not G.is_directed(),
                            depth_limit if depth_limit is not None else -1, True, False)
    df = pd.DataFrame({"vertex": vertex.cpu().numpy(), "predecessor": pred.cpu().numpy()})
    if return_distances:
        df.insert(1, "distance", d.cpu().numpy())
    return df


def sssp(input_graph, source, cutoff=None, check_source=True):
    """dask/traversal/sssp.py.  Returns this rank's rows of ['vertex', 'distance',
    'predecessor'] (distance float max and predecessor -1 when unreachable)."""
    import pandas as pd
    _check(input_graph)
    if not input_graph.is_weighted():
        raise ValueError("sssp needs a weighted graph (edge_attr)")
    p = _plc()
    h = _comms.get_default_handle()
    vertex, d, pred = p.sssp(h, input_graph._plc_graph, int(source), float("inf") if cutoff is None else cutoff,
                             True, False)
    return pd.DataFrame({"vertex": vertex.cpu().numpy(), "distance": d.cpu().numpy(),
                         "predecessor": pred.cpu().numpy()})


def louvain(input_graph, max_iter=100, resolution=1.0):
    """dask/community/louvain.py:53-161.  Returns (this rank's rows of ['vertex',
    'partition'], modularity) -- the same modularity on every rank."""
    import pandas as pd
    _check(input_graph)
    if input_graph.is_directed():
        raise ValueError("input graph must be undirected")
    p = _plc()
    h = _comms.get_default_handle()
    vertex, part, q = p.louvain(h, input_graph._weighted_plc_graph(), max_iter, resolution, False)
    return pd.DataFrame({"vertex": vertex.cpu().numpy(), "partition": part.cpu().numpy()}), q


def gather(df):
    """Every rank's partition of a result, concatenated (on every rank)."""
    import pandas as pd
    import torch.distributed as dist
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, df)
    return pd.concat(parts, ignore_index=True)


__all__ = ["pagerank", "bfs", "sssp", "louvain", "gather"]

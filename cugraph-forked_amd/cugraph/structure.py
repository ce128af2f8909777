"""cugraph.Graph / DiGraph (reference structure/graph_classes.py, simpleGraph.py)."""
from __future__ import annotations

import numpy as np


def _plc():
    import pylibcugraph
    return pylibcugraph


def _column(df, name):
    """A column of a pandas DataFrame / dict / anything indexable -> CUDA tensor."""
    import torch
    col = df[name]
    if isinstance(col, torch.Tensor):
        return col.cuda()
    if hasattr(col, "to_numpy"):
        col = col.to_numpy()
    return torch.as_tensor(np.ascontiguousarray(col)).cuda()


def _vertex_dtype(*cols):
    import torch
    hi = max((int(c.max().item()) for c in cols if c.numel()), default=0)
    lo = min((int(c.min().item()) for c in cols if c.numel()), default=0)
    if lo < 0:
        raise ValueError("vertex ids must be non-negative integers (renumbering of other ids is not supported)")
    return torch.int32 if hi < 2**31 - 1 else torch.int64


class Graph:
    """Undirected by default (graph_classes.py:63-65)."""

    class Properties:
        def __init__(self, directed):
            self.directed = directed
            self.weights = False

    def __init__(self, m_graph=None, directed=False):
        if m_graph is not None:
            raise TypeError("m_graph (MultiGraph conversion) is not supported by this build")
        self.graph_properties = Graph.Properties(directed)
        self._plc_graph = None
        self._plc_weighted = None
        self._handle = None
        self.edgelist = None
        self.renumbered = False
        self.store_transposed = False
        self._renumber = True

    # ------------------------------------------------------------ construction
    def from_cudf_edgelist(self, input_df, source="source", destination="destination", edge_attr=None,
                           renumber=True, store_transposed=False, legacy_renum_only=False):
        """graph_classes.py:95-171 -> simpleGraph.py:110-244."""
        if self.edgelist is not None:
            raise RuntimeError("Graph already has values")
        if isinstance(source, (list, tuple)) or isinstance(destination, (list, tuple)):
            raise ValueError("multi-column vertex ids are not supported by this build")
        cols = list(input_df.columns) if hasattr(input_df, "columns") else list(input_df.keys())
        if source not in cols or destination not in cols:
            raise ValueError("source column names and/or destination column names not found in input. "
                             "Recheck the source and destination parameters")
        if edge_attr is not None:
            if isinstance(edge_attr, (list, tuple)):
                if len(edge_attr) != 1:
                    raise ValueError(f"Invalid number of edge attributes passed. {edge_attr}")
                edge_attr = edge_attr[0]
            if edge_attr not in cols:
                raise ValueError("edge_attr column name not found in input.Recheck the edge_attr parameter")
        import torch
        src = _column(input_df, source)
        dst = _column(input_df, destination)
        if src.dtype not in (torch.int32, torch.int64) or dst.dtype not in (torch.int32, torch.int64):
            raise ValueError("set renumber to True for non integer columns ids" if not renumber else
                             "non-integer vertex ids are not supported by this build")
        vt = _vertex_dtype(src, dst)
        src, dst = src.to(vt), dst.to(vt)
        w = None
        if edge_attr is not None:
            w = _column(input_df, edge_attr)
            if w.dtype not in (torch.float32, torch.float64):
                w = w.to(torch.float32)
            self.graph_properties.weights = True
        p = _plc()
        self._handle = p.ResourceHandle()
        # symmetrize.py:78-93: reversed edges when undirected, duplicates dropped (min weight)
        src, dst, w = p.generators.symmetrize_dedup(self._handle, src, dst, w, not self.graph_properties.directed)
        self.edgelist = {"src": src, "dst": dst, "weights": w}
        self.store_transposed = bool(store_transposed)
        self._renumber = bool(renumber)
        self.renumbered = False  # ids stay external at the Python level; libcugraph_c renumbers
        self._plc_graph = self._make_plc_graph(w)

    def from_dask_cudf_edgelist(self, input_ddf, source="source", destination="destination", edge_attr=None,
                                renumber=True, store_transposed=False, legacy_renum_only=False):
        """graph_classes.py:173-244 -> simpleDistributedGraph.py.  One process per GPU:
        every rank calls this collectively with ITS partition of the edge list (a pandas
        DataFrame / dict of arrays or tensors); cugraph.dask.comms.comms.initialize()
        must have been called.  The partitions are symmetrised (undirected) and
        de-duplicated across the ranks (cugraph.dask._shuffle), then
        cugraph_mg_graph_create builds the 2D-partitioned graph."""
        import torch
        import torch.distributed as dist
        from .dask import _shuffle
        from .dask.comms import comms as dcomms
        if self.edgelist is not None:
            raise RuntimeError("Graph already has values")
        if not renumber:
            raise ValueError("the distributed graph is always renumbered (cugraph_mg_graph_create)")
        cols = list(input_ddf.columns) if hasattr(input_ddf, "columns") else list(input_ddf.keys())
        if source not in cols or destination not in cols:
            raise ValueError("source column names and/or destination column names not found in input. "
                             "Recheck the source and destination parameters")
        if isinstance(edge_attr, (list, tuple)):
            if len(edge_attr) != 1:
                raise ValueError(f"Invalid number of edge attributes passed. {edge_attr}")
            edge_attr = edge_attr[0]
        if edge_attr is not None and edge_attr not in cols:
            raise ValueError("edge_attr column name not found in input.Recheck the edge_attr parameter")
        h = dcomms.get_default_handle()
        src, dst = _column(input_ddf, source), _column(input_ddf, destination)
        w = None
        if edge_attr is not None:
            w = _column(input_ddf, edge_attr)
            if w.dtype not in (torch.float32, torch.float64):
                w = w.to(torch.float32)
            self.graph_properties.weights = True
        src, dst, w = _shuffle.shuffle_dedup(src, dst, w, self.graph_properties.directed)
        cdev = dcomms.collective_device()
        hi = torch.tensor([int(max(src.max(), dst.max())) if src.numel() else 0], dtype=torch.int64, device=cdev)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        vt = torch.int32 if int(hi) < 2**31 - 1 else torch.int64
        src, dst = src.to(vt), dst.to(vt)
        ne = torch.tensor([src.numel()], dtype=torch.int64, device=cdev)
        dist.all_reduce(ne)
        self.edgelist = {"src": src, "dst": dst, "weights": w}
        self.store_transposed = bool(store_transposed)
        self.renumbered = True
        self._handle = h
        self._distributed = True
        self._num_edges_global = int(ne)
        p = _plc()
        props = p.GraphProperties(is_symmetric=not self.graph_properties.directed, is_multigraph=False)
        self._plc_graph = p.MGGraph(h, props, src, dst, w, store_transposed=self.store_transposed,
                                    num_edges=self._num_edges_global)

    def from_pandas_edgelist(self, pdf, source="source", destination="destination", edge_attr=None,
                             renumber=True, store_transposed=False, legacy_renum_only=False):
        """graph_classes.py:295-350."""
        self.from_cudf_edgelist(pdf, source, destination, edge_attr, renumber, store_transposed, legacy_renum_only)

    def from_numpy_array(self, np_array, nodes=None):
        """graph_classes.py:368-395: dense adjacency -> weighted edge list."""
        import pandas as pd
        a = np.asarray(np_array)
        s, d = np.nonzero(a)
        df = pd.DataFrame({"source": s.astype(np.int64), "destination": d.astype(np.int64),
                           "weight": a[s, d].astype(np.float64)})
        self.from_pandas_edgelist(df, edge_attr="weight", renumber=nodes is None)

    def _make_plc_graph(self, weights):
        p = _plc()
        props = p.GraphProperties(is_symmetric=not self.graph_properties.directed, is_multigraph=False)
        e = self.edgelist
        return p.SGGraph(self._handle, props, e["src"], e["dst"], weights, store_transposed=self.store_transposed,
                         renumber=self._renumber, do_expensive_check=False)

    def _weighted_plc_graph(self):
        """simpleGraph.py:840-843 gives unweighted graphs all-ones fp32 weights; made on demand here."""
        if self.edgelist["weights"] is not None:
            return self._plc_graph
        if self._plc_weighted is None:
            import torch
            ones = torch.ones(self.edgelist["src"].numel(), dtype=torch.float32, device="cuda")
            if getattr(self, "_distributed", False):
                p = _plc()
                props = p.GraphProperties(is_symmetric=not self.graph_properties.directed, is_multigraph=False)
                self._plc_weighted = p.MGGraph(self._handle, props, self.edgelist["src"], self.edgelist["dst"], ones,
                                               store_transposed=self.store_transposed,
                                               num_edges=self._num_edges_global)
            else:
                self._plc_weighted = self._make_plc_graph(ones)
        return self._plc_weighted

    def is_distributed(self):
        return getattr(self, "_distributed", False)

    # ------------------------------------------------------------ queries
    def is_directed(self):
        return self.graph_properties.directed

    def is_weighted(self):
        return self.graph_properties.weights

    def is_renumbered(self):
        return self.renumbered

    def is_multigraph(self):
        return False

    def number_of_vertices(self):
        return self._plc_graph.number_of_vertices()

    def number_of_nodes(self):
        return self.number_of_vertices()

    def number_of_edges(self, directed_edges=False):
        n = self._plc_graph.number_of_edges()
        return n if (directed_edges or self.is_directed()) else n // 2

    def view_edge_list(self):
        import pandas as pd
        e = self.edgelist
        s, d = e["src"].cpu().numpy(), e["dst"].cpu().numpy()
        cols = {"src": s, "dst": d}
        if e["weights"] is not None:
            cols["weights"] = e["weights"].cpu().numpy()
        df = pd.DataFrame(cols)
        if not self.is_directed():  # the undirected edge list is stored symmetrised: one row per edge
            df = df[df["src"] <= df["dst"]].reset_index(drop=True)
        return df

    def nodes(self):
        import torch
        e = self.edgelist
        return torch.unique(torch.cat([e["src"], e["dst"]])).cpu().numpy()

    def has_node(self, n):
        e = self.edgelist
        return bool(((e["src"] == n).any() | (e["dst"] == n).any()).item())

    def to_undirected(self):
        G = Graph()
        import pandas as pd
        e = self.edgelist
        cols = {"src": e["src"].cpu().numpy(), "dst": e["dst"].cpu().numpy()}
        if e["weights"] is not None:
            cols["w"] = e["weights"].cpu().numpy()
        G.from_pandas_edgelist(pd.DataFrame(cols), "src", "dst", "w" if "w" in cols else None, self._renumber,
                               self.store_transposed)
        return G


class DiGraph(Graph):
    def __init__(self, m_graph=None):
        super().__init__(m_graph=m_graph, directed=True)


def from_edgelist(df, source="source", destination="destination", edge_attr=None, create_using=Graph,
                  renumber=True):
    G = create_using() if isinstance(create_using, type) else create_using
    G.from_cudf_edgelist(df, source, destination, edge_attr, renumber)
    return G


def from_pandas_edgelist(df, source="source", destination="destination", edge_attr=None, create_using=Graph,
                         renumber=True):
    G = create_using() if isinstance(create_using, type) else create_using
    G.from_pandas_edgelist(df, source, destination, edge_attr, renumber)
    return G

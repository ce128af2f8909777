"""cugraph-compatible Python API over the MI355X libcugraph_c (hot path only).

Mirrors the reference's ``python/cugraph/cugraph`` surface for PageRank, BFS,
SSSP and Louvain: ``Graph`` / ``DiGraph`` with ``from_cudf_edgelist`` semantics
(structure/graph_classes.py:95-171, graph_implementation/simpleGraph.py:110-244:
symmetrise when undirected, drop duplicate edges keeping the minimum weight,
renumber in libcugraph_c), and the algorithm wrappers with their argument names,
defaults, result columns and NetworkX-graph handling.  cudf is not available in
this image: edge lists are pandas DataFrames (or dicts of numpy arrays / torch
tensors) and results come back as pandas DataFrames.
"""
from .structure import DiGraph, Graph, from_edgelist, from_pandas_edgelist
from .algorithms import (bfs, eigenvector_centrality, hits, katz_centrality, louvain, pagerank, shortest_path,
                         shortest_path_length, sssp)
from . import generators
from . import dask  # noqa: F401  (multi-GPU, one process per GPU)

__all__ = ["Graph", "DiGraph", "from_edgelist", "from_pandas_edgelist", "pagerank", "bfs", "sssp",
           "shortest_path", "shortest_path_length", "louvain", "katz_centrality", "eigenvector_centrality", "hits",
           "generators", "dask"]

"""Helpers for the -m gpu parity tests (everything goes through the C ABI via the
pylibcugraph shim; the oracle only checks)."""
import numpy as np


def plc():
    import pylibcugraph
    return pylibcugraph


def make_graph(src, dst, w=None, transposed=False, renumber=True, symmetric=False, vdtype=np.int32,
               wdtype=np.float32, handle=None, options=None):
    """options: measurement / A-B switches set on the new handle (set_option,
    include/cugraph_amd/ext.h) before the graph is built."""
    p = plc()
    h = handle or p.ResourceHandle()
    for k, v in (options or {}).items():
        h.set_option(k, v)
    props = p.GraphProperties(is_symmetric=symmetric, is_multigraph=False)
    s = np.asarray(src, dtype=vdtype)
    d = np.asarray(dst, dtype=vdtype)
    ww = None if w is None else np.asarray(w, dtype=wdtype)
    g = p.SGGraph(h, props, s, d, ww, store_transposed=transposed, renumber=renumber)
    return h, g


def host(t):
    return t.cpu().numpy()


def ext_to_int_map(vertices):
    """dict external id -> position in the result arrays."""
    v = host(vertices)
    return {int(x): i for i, x in enumerate(v)}

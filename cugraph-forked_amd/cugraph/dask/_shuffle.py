"""Distributed edge-list preprocessing for ``Graph.from_dask_cudf_edgelist``
(reference ``structure/graph_implementation/simpleDistributedGraph.py``:
``symmetrize_ddf`` then ``drop_duplicates`` over the dask DataFrame).

Every rank passes its partition of the edge list.  Edges are sent to the rank that
owns their (canonical, for undirected graphs) pair under a hash, with one
``torch.distributed.all_to_all_single`` per column; the owner drops duplicates
keeping the minimum weight (symmetrize.py:78-93 keeps the min) and, for an
undirected graph, emits both directions.  The union over the ranks is then the
reference's symmetrised, de-duplicated edge list, split over the ranks.
"""
from __future__ import annotations


def _owner(a, b, P):
    import torch
    h = (a * 0x9E3779B1 + b * 0x85EBCA77) & ((1 << 62) - 1)
    h = h ^ (h >> 29)
    return torch.remainder(h, P)


def _exchange(t, dest, P, group=None):
    """Rows of t (1-D tensor) to rank dest[i]; returns the received rows."""
    import torch
    import torch.distributed as dist
    order = torch.argsort(dest, stable=True)
    t = t[order]
    send = torch.bincount(dest, minlength=P)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    out = torch.empty(int(recv.sum()), dtype=t.dtype, device=t.device)
    dist.all_to_all_single(out, t.contiguous(), output_split_sizes=recv.tolist(),
                           input_split_sizes=send.tolist(), group=group)
    return out


def shuffle_dedup(src, dst, w, directed):
    """(src, dst, w) of this rank (CUDA or CPU tensors) -> this rank's share of the
    global edge list after symmetrisation (undirected) and de-duplication."""
    import torch
    import torch.distributed as dist
    P = dist.get_world_size()
    dev = src.device
    from .comms.comms import collective_device
    s, d = src.to(torch.int64), dst.to(torch.int64)
    if not directed:  # canonical pair: the smaller id first
        s, d = torch.minimum(s, d), torch.maximum(s, d)
    cdev = collective_device()
    s, d = s.to(cdev), d.to(cdev)
    w = None if w is None else w.to(cdev)
    dest = _owner(s, d, P)
    s, d = _exchange(s, dest, P), _exchange(d, dest, P)
    ww = None if w is None else _exchange(w, dest, P)
    # local de-duplication, minimum weight
    n = int(max(int(s.max()) if s.numel() else 0, int(d.max()) if d.numel() else 0)) + 1
    key = s * n + d
    uk, inv = torch.unique(key, return_inverse=True)
    s, d = uk // n, uk % n
    if ww is not None:
        mw = torch.full((uk.numel(),), float("inf"), dtype=ww.dtype, device=ww.device)
        ww = mw.scatter_reduce(0, inv, ww, reduce="amin")
    if not directed:  # both directions (self loops once)
        off = s != d
        s, d = torch.cat([s, d[off]]), torch.cat([d, s[off]])
        if ww is not None:
            ww = torch.cat([ww, ww[off]])
    return s.to(dev), d.to(dev), None if ww is None else ww.to(dev)

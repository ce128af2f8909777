"""cugraph.dask edge-list preprocessing on CPU (gloo, world sizes 2 and 3): each rank
holds a partition with duplicates inside and across the partitions; after
cugraph.dask._shuffle.shuffle_dedup the union over the ranks must be exactly the
symmetrised, de-duplicated (minimum weight) edge list of the oracle
(oracle/graph.py symmetrize_dedup, the reference's symmetrize.py:78-93), each edge
on one rank only."""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _edges(seed=3, n=400, V=60):
    rng = np.random.default_rng(seed)
    s = rng.integers(0, V, n)
    d = rng.integers(0, V, n)
    w = rng.random(n)
    # explicit duplicates (also reversed) with different weights
    s = np.concatenate([s, d[:50], s[:30]])
    d = np.concatenate([d, s[:50], d[:30]])
    w = np.concatenate([w, w[:50] + 0.5, w[:30] - 0.25])
    return s, d, w


def _worker(rank, world, port, directed, weighted, q):
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cugraph.dask import _shuffle
    s, d, w = _edges()
    part = np.arange(rank, s.size, world)  # an uneven interleaved split
    st, dt = torch.as_tensor(s[part]), torch.as_tensor(d[part])
    wt = torch.as_tensor(w[part]) if weighted else None
    rs, rd, rw = _shuffle.shuffle_dedup(st, dt, wt, directed)
    q.put((rank, rs.numpy(), rd.numpy(), None if rw is None else rw.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,directed,weighted", [(2, False, True), (3, True, True), (2, False, False)])
def test_shuffle_dedup_matches_oracle(world, directed, weighted):
    pytest.importorskip("torch")
    import torch.multiprocessing as tmp
    sys.path.insert(0, ROOT)
    from oracle import graph as og
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, directed, weighted, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s, d, w = _edges()
    es, ed, ew = og.symmetrize_dedup(s, d, w if weighted else None, symmetrize=not directed)
    got = {}
    for _, rs, rd, rw in res:
        for i in range(rs.size):
            key = (int(rs[i]), int(rd[i]))
            assert key not in got, "an edge on two ranks"
            got[key] = None if rw is None else float(rw[i])
    want = {(int(a), int(b)): (None if ew is None else float(c)) for a, b, c in
            zip(es, ed, ew if ew is not None else [None] * es.size)}
    assert got == want

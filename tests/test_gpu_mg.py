"""Multi-GPU path (cugraph_mg_graph_create + MG PageRank / BFS / SSSP / Louvain) on ONE
MI355X: 1-4 ranks share cuda:0 and talk through torch.distributed/gloo callbacks
(pylibcugraph.comms.init_torch) -- RCCL refuses two ranks per GPU.  The 2D
partition, the id routing and the per-iteration collectives are the same code as
with RCCL; results are checked against the single-GPU oracle."""
import os
import socket

import numpy as np
import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _slice(rank, world, E):
    """This rank's slice of the edge list.  CGX_TEST_SKEW=1: rank 0 passes no edges
    at all and the others split the list (ranks whose input is empty)."""
    if os.environ.get("CGX_TEST_SKEW") and world > 1:
        if rank == 0:
            return 0, 0
        return (rank - 1) * E // (world - 1), rank * E // (world - 1)
    return rank * E // world, (rank + 1) * E // world


def _stack_file(port, rank):
    return f"/tmp/cgx_stacks_{port}_{rank}.txt"


def _rank_setup(port=None, rank=None):
    """In a worker, before its first HIP call:
    * SIGUSR1 writes every thread's stack (from the signal handler, so a rank blocked
      inside a C call still answers) to the rank's own file, which _spawn prints rank
      by rank on a deadline (8 ranks writing one stderr interleaved their stacks
      beyond reading);
    * HSA_ENABLE_SDMA=0: copies run as blit kernels, not on the DMA engines.  Up to 8
      rehearsal ranks share the one test GPU, and the world-8 Louvain rehearsal (the
      most copy-heavy: hundreds of small staged collectives per rank) stalled in 3 of
      5 round-3 runs: the stacks show every arrived rank inside the same collective and
      the missing ones blocked draining their own stream's copies ("The
      world-8 rehearsal hang").  A node runs one rank per GPU over RCCL instead."""
    import faulthandler
    import signal
    import sys
    os.environ.setdefault("HSA_ENABLE_SDMA", "0")
    out = sys.stderr if port is None else open(_stack_file(port, rank), "w")
    faulthandler.register(signal.SIGUSR1, file=out, all_threads=True)


def _spawn(fn, args, nprocs, deadline=150.0):
    """torch.multiprocessing.spawn with a deadline: on expiry every live rank prints
    its stacks (SIGUSR1, see _rank_setup), all ranks are killed and the test
    fails naming them -- one hung rehearsal does not take the suite down with it."""
    import signal
    import time
    import torch.multiprocessing as tmp
    ctx = tmp.start_processes(fn, args=args, nprocs=nprocs, join=False, start_method="spawn")
    end = time.monotonic() + deadline
    while time.monotonic() < end:
        if ctx.join(timeout=1.0):
            return
    alive = [r for r, p in enumerate(ctx.processes) if p.is_alive()]
    for r in alive:
        try:
            os.kill(ctx.processes[r].pid, signal.SIGUSR1)
        except OSError:
            pass
    time.sleep(3.0)
    port = args[1]
    for r in alive:
        try:
            print(f"===== rank {r} stacks =====\n" + open(_stack_file(port, r)).read(), flush=True)
        except OSError:
            print(f"===== rank {r}: no stack file", flush=True)
    for p in ctx.processes:
        if p.is_alive():
            p.kill()
    for p in ctx.processes:
        p.join(10)
    pytest.fail(f"ranks {alive} of {nprocs} still running after {deadline:.0f} s (stacks above)")


def _graph(scale, weighted, seed=5):
    """RMAT(scale, 16) symmetrised; scale = -k: RMAT(k) with a path of 300 new
    vertices hung from vertex 1 (a long tail of one-vertex frontiers while most of the
    path is unvisited: the MG BFS returns to top-down, mg_bfs.hip kTdBack)."""
    from oracle import graph as og
    from oracle import rmat
    if scale < 0:
        s, d = rmat.rmat(-scale, 16 << -scale, seed=seed)
        n0 = 1 << -scale
        chain = np.arange(n0, n0 + 300, dtype=s.dtype)
        s = np.concatenate([s, np.array([1], s.dtype), chain[:-1]])
        d = np.concatenate([d, chain[:1], chain[1:]])
        w = rmat.rmat_weights(s.size, seed=seed + 1).astype(np.float64) if weighted else None
        return og.symmetrize_dedup(s, d, w)
    s, d = rmat.rmat(scale, 16 << scale, seed=seed)
    w = rmat.rmat_weights(s.size, seed=seed + 1).astype(np.float64) if weighted else None
    return og.symmetrize_dedup(s, d, w)


def _worker(rank, world, port, C, scale, weighted, algo, comm="torch"):
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _rank_setup(port, rank)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pylibcugraph as plc
    from oracle import graph as og
    from oracle import pagerank as opr
    from oracle import bfs as obfs

    s, d, w = _graph(scale, weighted)
    E = s.size
    lo, hi = _slice(rank, world, E)
    ctx = plc.comms.init_torch(C) if comm == "torch" else plc.comms.init_rccl(C)
    h = plc.ResourceHandle(ctx.ptr)
    assert h.get_rank() == rank
    st = torch.as_tensor(s[lo:hi].astype(np.int32), device="cuda")
    dt = torch.as_tensor(d[lo:hi].astype(np.int32), device="cuda")
    wt = None if w is None else torch.as_tensor(w[lo:hi].astype(np.float32), device="cuda")
    G = plc.MGGraph(h, plc.GraphProperties(is_symmetric=True, is_multigraph=False), st, dt, wt,
                    store_transposed=(algo == "pagerank"), num_edges=E)
    V = int(np.unique(np.concatenate([s, d])).size)
    assert G.number_of_vertices() == V and G.number_of_edges() == E
    if algo == "pagerank":
        v, x = plc.pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        mine = (v.cpu().numpy(), x.cpu().numpy())
        # the first call re-dealt this rank's push queues by measured item cost
        # (pagerank.hip calibrate_queues): a second call on them gives the same bits
        v2, x2 = plc.pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        assert np.array_equal(v2.cpu().numpy(), mine[0]) and np.array_equal(x2.cpu().numpy(), mine[1])
    else:
        root = int(np.unique(s)[0])
        src = np.array([root], np.int64) if rank == world - 1 else np.zeros(0, np.int64)
        srct = torch.as_tensor(src.astype(np.int32), device="cuda")
        dist_, pred, v = plc.bfs(h, G, srct, algo == "bfs_do", 0, True, False)
        mine = (v.cpu().numpy(), dist_.cpu().numpy(), pred.cpu().numpy())
        if scale < 0:  # the long tail: bottom-up levels in the core, then top-down ones again
            lv, bu = h.last_bfs_levels(), h.last_bfs_bottom_up_steps()
            assert bu > 0 and lv - bu > 250, (lv, bu)
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        verts = np.concatenate([a[0] for a in allr])
        assert np.array_equal(np.sort(verts), np.unique(np.concatenate([s, d])))  # each vertex exactly once
        ww = None if w is None else w.astype(np.float32).astype(np.float64)
        if algo == "pagerank":
            vals = np.concatenate([a[1] for a in allr])
            g = og.create_graph(s, d, ww, store_transposed=True, renumber=True)
            ref = opr.pagerank_from_graph(g, alpha=0.85, epsilon=1e-6, max_iterations=500)
            ref_ext = np.zeros(int(g.number_map.max()) + 1)
            ref_ext[g.number_map] = ref
            rel = np.abs(vals - ref_ext[verts]) / ref_ext[verts]
            assert rel.max() < 1e-6, rel.max()
        else:
            dists = np.concatenate([a[1] for a in allr])
            preds = np.concatenate([a[2] for a in allr])
            n = int(max(s.max(), d.max())) + 1
            g = og.create_graph(s, d, None, store_transposed=False, renumber=False, vertices=np.arange(n))
            root = int(np.unique(s)[0])
            rd, _ = obfs.bfs(g.num_vertices, g.offsets, g.indices, [root])
            assert np.array_equal(dists, rd[verts])  # bit-exact distances
            # predecessors valid (cpp/tests/traversal/mg_bfs_test.cpp rule): dist[p] + 1 == dist[v], edge p-v
            reached = (dists != 2**31 - 1) & (verts != root)
            pv = preds[reached]
            assert np.array_equal(rd[pv] + 1, dists[reached])
            adj = set(zip(s.tolist(), d.tolist()))
            assert all((int(p_), int(v_)) in adj for p_, v_ in zip(pv, verts[reached]))
            assert np.all(preds[~reached] == -1)
    dist.barrier()
    h = None
    G = None
    ctx.free()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,C,weighted", [(2, 2, False), (4, 2, True), (2, 1, False)])
def test_mg_pagerank_vs_oracle(world, C, weighted):
    _spawn(_worker, (world, _free_port(), C, 11, weighted, "pagerank"), world)


@pytest.mark.parametrize("world,C,algo", [(2, 2, "bfs"), (4, 2, "bfs_do"), (3, 3, "bfs_do"), (2, 1, "bfs"),
                                          (4, 1, "bfs_do")])
def test_mg_bfs_vs_oracle(world, C, algo):
    _spawn(_worker, (world, _free_port(), C, 12, False, algo), world)


@pytest.mark.parametrize("world,C", [(2, 2), (4, 2)])
def test_mg_bfs_long_tail_returns_to_top_down(world, C):
    """Direction-optimising MG BFS on RMAT-10 plus a 300-vertex path: bottom-up in the
    core, then back to top-down for the path (most of it unvisited), distances exact
    and predecessors valid (mg_bfs_test.cpp rule)."""
    _spawn(_worker, (world, _free_port(), C, -10, False, "bfs_do"), world)


@pytest.mark.parametrize("algo", ["pagerank", "bfs_do"])
def test_mg_rccl_single_rank(algo):
    """The RCCL communicators themselves (world / split row / split column), with the
    one rank a single GPU allows: every collective of the MG path runs through RCCL."""
    _spawn(_worker, (1, _free_port(), 1, 11, False, algo, "rccl"), 1)


def _same_partition(a, b):
    """renumbered_vectors_same (cpp/tests/utilities): equal up to a relabelling."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    pairs = np.unique(np.stack([a, b]), axis=1).shape[1]
    return pairs == np.unique(a).size == np.unique(b).size


def _louvain_worker(rank, world, port, C, scale, integer, comm="torch"):
    """MG Louvain checked as cpp/tests/community/mg_louvain_test.cpp:82-151 does:
    the SG algorithm (here the oracle) on the graph renumbered by the MG number map
    reproduces every MG dendrogram level as a partition, the SG graph is coarsened
    by the MG level, and the final modularities agree."""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _rank_setup(port, rank)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pylibcugraph as plc
    from oracle import graph as og
    from oracle import louvain as olv
    from oracle import rmat

    s, d = rmat.rmat(scale, 16 << scale, seed=7)
    w = rmat.rmat_weights(s.size, seed=8).astype(np.float64)
    if integer:
        w = np.floor(w * 8.0) + 1.0
    s, d, w = og.symmetrize_dedup(s, d, w)
    w = w.astype(np.float32).astype(np.float64)
    E = s.size
    lo, hi = _slice(rank, world, E)
    ctx = plc.comms.init_torch(C) if comm == "torch" else plc.comms.init_rccl(C)
    h = plc.ResourceHandle(ctx.ptr)
    st = torch.as_tensor(s[lo:hi].astype(np.int32), device="cuda")
    dt = torch.as_tensor(d[lo:hi].astype(np.int32), device="cuda")
    wt = torch.as_tensor(w[lo:hi].astype(np.float32), device="cuda")
    G = plc.MGGraph(h, plc.GraphProperties(is_symmetric=True, is_multigraph=False), st, dt, wt,
                    store_transposed=False, num_edges=E)
    v, c, q, levels = plc.louvain_dendrogram(h, G, 100, 1.0)
    # owner-sharded state: per-sweep exchange volume (sends to other ranks only)
    sb = h.last_louvain_sweep_bytes()
    part = h.last_louvain_partition()  # (level-0 edges, ghosts) of this rank's 1D share
    mine = (v.cpu().numpy(), c.cpu().numpy(), q, [x.cpu().numpy() for x in levels], sb, part)
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:  # (every check after the gather: a rank that failed alone would hang the others)
        for a in allr:
            assert (a[4] > 0) if world > 1 else (a[4] == 0), a[4]
            assert a[4] < 64 * E / world + 4096, a[4]  # O(moved + referenced) per sweep, not O(V)
        assert all(a[2] == q for a in allr)  # every rank returns the same modularity
        # the 1D partition: every edge at the owner of its source; report the shape
        assert sum(a[5][0] for a in allr) == E, [a[5] for a in allr]
        if world > 1:
            print(f"RMAT-{scale} MG Louvain {world} ranks: level-0 edges per rank {[a[5][0] for a in allr]} "
                  f"(E={E}), ghosts per rank {[a[5][1] for a in allr]} (V={int(np.unique(np.concatenate([s, d])).size)})")
        nmap = np.concatenate([a[0] for a in allr]).astype(np.int64)  # global id -> external id
        assert np.array_equal(np.sort(nmap), np.unique(np.concatenate([s, d])))
        inv = np.zeros(int(nmap.max()) + 1, dtype=np.int64)
        inv[nmap] = np.arange(nmap.size)
        L = len(levels)
        lv = [np.concatenate([a[3][i] for a in allr]).astype(np.int64) for i in range(L)]
        gs, gd, gw, V = inv[s], inv[d], w, nmap.size
        best, qs = -1.0, []
        for i in range(L):
            assert lv[i].size == V
            oc, oq, _ = olv.louvain(V, gs, gd, gw, max_level=1)
            if integer:
                assert _same_partition(oc, lv[i]), f"level {i}"
            qs.append(oq)
            if oq <= best:
                assert i == L - 1, "MG went on after a level without gain"
                break
            best = oq
            if i + 1 < L:  # coarsen the SG graph by the MG level (mg_louvain_helper coarsen_graph)
                cs, cd = lv[i][gs], lv[i][gd]
                key = cs * (lv[i].max() + 1) + cd
                uk, inv_k = np.unique(key, return_inverse=True)
                gw = np.bincount(inv_k, weights=gw)
                gs, gd = uk // (lv[i].max() + 1), uk % (lv[i].max() + 1)
                V = lv[i + 1].size
        if integer:
            assert q == pytest.approx(best, rel=1e-12, abs=1e-12)
        else:
            assert q == pytest.approx(best, rel=1e-6)
        # the flattened clustering is the composition of the levels
        flat = np.arange(nmap.size)
        for x in lv:
            flat = x[flat]
        clus = np.concatenate([a[1] for a in allr]).astype(np.int64)
        assert np.array_equal(clus, flat)
        assert olv.modularity(inv[s], inv[d], w, flat) >= q - 1e-9
        if world == 1 and integer:  # one rank: exactly the single-GPU algorithm
            OG = og.create_graph(s, d, w, renumber=True)
            os_, od, ow = OG.coo()
            oc, oq, olevels = olv.louvain(OG.num_vertices, os_, od, ow, 100, 1.0)
            assert np.array_equal(OG.number_map, nmap) and np.array_equal(oc, clus)
            assert q == oq and olevels == L
    dist.barrier()
    h = None
    G = None
    ctx.free()
    dist.destroy_process_group()


def _louvain_negative_worker(rank, world, port, C):
    """A negative edge weight: MG Louvain's owner-side fixed-point cluster weights assume
    w >= 0, so every rank must refuse the graph with the same error (no rank may go on
    into a collective the others skip)."""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _rank_setup(port, rank)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pylibcugraph as plc
    s, d, w = _graph(8, True)
    w = w.astype(np.float32)
    w[5] = -0.5  # one entry only (the graph is no longer symmetric in w: irrelevant here)
    E = s.size
    lo, hi = _slice(rank, world, E)
    ctx = plc.comms.init_torch(C)
    h = plc.ResourceHandle(ctx.ptr)
    dev = lambda a, t: torch.as_tensor(np.ascontiguousarray(a).astype(t), device="cuda")  # noqa: E731
    G = plc.MGGraph(h, plc.GraphProperties(is_symmetric=True, is_multigraph=False), dev(s[lo:hi], np.int32),
                    dev(d[lo:hi], np.int32), dev(w[lo:hi], np.float32), store_transposed=False, num_edges=E)
    with pytest.raises(RuntimeError, match="negative"):
        plc.louvain(h, G, 100, 1.0, False)
    dist.barrier()
    h = None
    G = None
    ctx.free()
    dist.destroy_process_group()


def test_mg_louvain_negative_weight_refused():
    _spawn(_louvain_negative_worker, (2, _free_port(), 2), 2)


@pytest.mark.parametrize("world,C,integer", [(2, 2, True), (3, 3, True), (4, 2, True), (2, 1, False)])
def test_mg_louvain_levels_vs_oracle(world, C, integer):
    _spawn(_louvain_worker, (world, _free_port(), C, 10, integer), world)


def test_mg_louvain_rccl_single_rank():
    _spawn(_louvain_worker, (1, _free_port(), 1, 11, True, "rccl"), 1)


def _pr_options_worker(rank, world, port, C):
    """MG personalized PageRank with an initial guess and precomputed out-weight sums,
    each (vertex, value) list split unevenly over the ranks (the reference shuffles
    such pairs to their owners, c_api/pagerank.cpp MG branch), vs the oracle."""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _rank_setup(port, rank)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pylibcugraph as plc
    from oracle import graph as og
    from oracle import pagerank as opr

    s, d, w = _graph(10, True)
    w = w.astype(np.float32).astype(np.float64)
    E = s.size
    lo, hi = _slice(rank, world, E)
    ctx = plc.comms.init_torch(C)
    h = plc.ResourceHandle(ctx.ptr)
    dev = lambda a, t: torch.as_tensor(np.ascontiguousarray(a).astype(t), device="cuda")  # noqa: E731
    G = plc.MGGraph(h, plc.GraphProperties(is_symmetric=True, is_multigraph=False), dev(s[lo:hi], np.int32),
                    dev(d[lo:hi], np.int32), dev(w[lo:hi], np.float32), store_transposed=True, num_edges=E)
    verts = np.unique(np.concatenate([s, d]))
    outw = np.zeros(int(verts.max()) + 1)
    np.add.at(outw, s, w)
    rng = np.random.default_rng(3)
    pv = rng.choice(verts, 40, replace=False)
    pval = rng.random(40) + 0.1
    gv = rng.choice(verts, 200, replace=False)
    gval = rng.random(200) + 0.5
    mine = lambda a: a[rank::world] if rank < world - 1 else a[rank::world][:3]  # noqa: E731
    ow_v = verts if rank == 0 else verts[:0]  # all out-weights given by rank 0
    v, x = plc.personalized_pagerank(
        h, G, dev(ow_v, np.int32), dev(outw[ow_v], np.float32), dev(mine(gv), np.int32),
        dev(mine(gval), np.float32), dev(mine(pv), np.int32), dev(mine(pval), np.float32), 0.85, 1e-6, 500, True)
    res = (v.cpu().numpy(), x.cpu().numpy(), mine(pv), mine(pval), mine(gv), mine(gval))
    allr = [None] * world
    dist.all_gather_object(allr, res)
    if rank == 0:
        vv = np.concatenate([a[0] for a in allr])
        xx = np.concatenate([a[1] for a in allr])
        pv_all = np.concatenate([a[2] for a in allr])
        pval_all = np.concatenate([a[3] for a in allr]).astype(np.float32).astype(np.float64)
        g = og.create_graph(s, d, w, store_transposed=True, renumber=True)
        inv = np.zeros(int(g.number_map.max()) + 1, dtype=np.int64)
        inv[g.number_map] = np.arange(g.number_map.size)
        guess = np.zeros(g.number_map.size)
        guess[inv[np.concatenate([a[4] for a in allr])]] = np.concatenate([a[5] for a in allr]).astype(np.float32)
        ref = opr.pagerank_from_graph(g, alpha=0.85, epsilon=1e-6, max_iterations=500, initial_guess=guess,
                                      personalization_vertices=inv[pv_all], personalization_values=pval_all)
        got = np.zeros(g.number_map.size)
        got[inv[vv]] = xx
        live = ref > 1e-9
        rel = np.abs(got - ref)[live] / ref[live]
        assert rel.max() < 1e-6, rel.max()
    dist.barrier()
    h = None
    G = None
    ctx.free()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,C", [(2, 2), (3, 1)])
def test_mg_personalized_pagerank_options(world, C):
    _spawn(_pr_options_worker, (world, _free_port(), C), world)


def _sssp_worker(rank, world, port, C, scale, symmetric, cutoff):
    """MG SSSP vs the oracle's fp32 min-plus fixed point: distances bit-identical,
    predecessors = the tight in-neighbour with the smallest global id (the oracle's
    tie_key set to the MG global order)."""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _rank_setup(port, rank)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pylibcugraph as plc
    from oracle import graph as og
    from oracle import rmat
    from oracle import sssp as osssp

    s, d = rmat.rmat(scale, 16 << scale, seed=11)
    w = rmat.rmat_weights(s.size, seed=43).astype(np.float64)
    s, d, w = og.symmetrize_dedup(s, d, w, symmetrize=symmetric)
    E = s.size
    lo, hi = _slice(rank, world, E)
    ctx = plc.comms.init_torch(C)
    h = plc.ResourceHandle(ctx.ptr)
    dev = lambda a, t: torch.as_tensor(np.ascontiguousarray(a).astype(t), device="cuda")  # noqa: E731
    G = plc.MGGraph(h, plc.GraphProperties(is_symmetric=symmetric, is_multigraph=False), dev(s[lo:hi], np.int32),
                    dev(d[lo:hi], np.int32), dev(w[lo:hi], np.float32), store_transposed=False, num_edges=E)
    src = int(s[0])
    v, dd, pp = plc.sssp(h, G, src, cutoff, True, True)
    allr = [None] * world
    dist.all_gather_object(allr, (v.cpu().numpy(), dd.cpu().numpy(), pp.cpu().numpy()))
    if rank == 0:
        vv = np.concatenate([a[0] for a in allr])  # global id order
        dv = np.concatenate([a[1] for a in allr])
        pv = np.concatenate([a[2] for a in allr])
        n_ext = int(max(s.max(), d.max())) + 1
        G2 = og.create_graph(s, d, w.astype(np.float32), renumber=False, vertices=np.arange(n_ext))
        key = np.empty(n_ext, np.int64)  # a permutation: graph vertices in global order, then absent ids
        key[vv] = np.arange(vv.size)
        absent = np.setdiff1d(np.arange(n_ext), vv)
        key[absent] = vv.size + np.arange(absent.size)
        rd, rp = osssp.sssp(n_ext, G2.offsets, G2.indices, G2.weights, src, cutoff=cutoff, tie_key=key)
        assert np.array_equal(dv, rd[vv])
        assert np.array_equal(pv, rp[vv])
    dist.barrier()
    h = None
    G = None
    ctx.free()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,C,symmetric,cutoff", [(2, 2, True, np.inf), (3, 3, False, np.inf),
                                                       (4, 2, True, 0.05)])
def test_mg_sssp_vs_oracle(world, C, symmetric, cutoff):
    _spawn(_sssp_worker, (world, _free_port(), C, 11, symmetric, float(cutoff)), world)


@pytest.mark.parametrize("algo", ["pagerank", "bfs_do", "louvain", "sssp"])
def test_mg_rank_without_edges(algo, monkeypatch):
    """Rank 0 contributes no edges to cugraph_mg_graph_create (it still owns vertices)."""
    monkeypatch.setenv("CGX_TEST_SKEW", "1")
    port = _free_port()
    if algo == "louvain":
        _spawn(_louvain_worker, (3, port, 3, 10, True), 3)
    elif algo == "sssp":
        _spawn(_sssp_worker, (3, port, 3, 10, True, float("inf")), 3)
    else:
        _spawn(_worker, (3, port, 3, 10, False, algo), 3)


# The reference's 8-GPU grid (mg_utilities.cpp:59-62: row communicator size = the
# largest divisor of 8 not above sqrt(8) = 2, so R x C = 4 x 2 -- bench.py's default at
# N = 8) and its transpose 2 x 4, rehearsed with 8 ranks on the one test GPU over
# torch.distributed/gloo: the same partition, id routing and per-level /
# per-iteration collectives an 8 x MI355X node runs over RCCL (performance
# unmeasured here).
@pytest.mark.parametrize("algo,C", [("pagerank", 2), ("pagerank", 4), ("bfs_do", 2), ("bfs_do", 4), ("bfs", 2),
                                    ("bfs", 4), ("louvain", 2)])
def test_mg_world8_reference_grid(algo, C):
    """(Louvain is partitioned 1D by source owner whatever the grid: only the
    reference's 4 x 2 build is rehearsed for it.)"""
    port = _free_port()
    if algo == "louvain":
        _spawn(_louvain_worker, (8, port, C, 10, True), 8)
    else:
        _spawn(_worker, (8, port, C, 11, False, algo), 8)


def _mg_sg_worker(rank, world, port, C, scale, chunks=None):
    """MG against the single-GPU library on the same graph (the reference's MG tests:
    cpp/tests/link_analysis/mg_pagerank_test.cpp:258-270,333-347 compares MG with SG
    on RMAT(20, 32); cpp/tests/traversal/mg_bfs_test.cpp:160-225):
    * PageRank bit for bit per external id, same iteration count -- the push sums are
      u64 fixed point and the (diff, dangling) totals are allreduced as u64, so the
      partition changes no bit;
    * BFS (direction-optimising) distances equal to SG's;
    * BFS predecessors equal to SG's on the graph renumbered by the MG number map (the
      reference's MG-test method, mg_louvain_test.cpp:69-90): both take the frontier
      neighbour with the smallest id, and with the MG numbering those ids agree.
      (On SG's own numbering the predecessor is another valid parent, checked by
      tests/test_gpu_bench_parity.py's rule.)"""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _rank_setup(port, rank)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pylibcugraph as plc

    s, d, _ = _graph(scale, False, seed=17)
    E = s.size
    lo, hi = _slice(rank, world, E)
    ctx = plc.comms.init_torch(C)
    h = plc.ResourceHandle(ctx.ptr)
    if chunks:
        h.set_option("mg_chunks", chunks)
    props = plc.GraphProperties(is_symmetric=True, is_multigraph=False)
    dev = lambda a: torch.as_tensor(np.ascontiguousarray(a).astype(np.int32), device="cuda")  # noqa: E731
    Gp = plc.MGGraph(h, props, dev(s[lo:hi]), dev(d[lo:hi]), None, store_transposed=True, num_edges=E)
    v, x = plc.pagerank(h, Gp, None, None, None, None, 0.85, 1e-6, 500, False)
    it = h.last_iterations()
    Gp = None
    Gb = plc.MGGraph(h, props, dev(s[lo:hi]), dev(d[lo:hi]), None, store_transposed=False, num_edges=E)
    root = int(s[np.argmax(np.bincount(s))])  # a hub: the traversal switches to bottom-up early
    srct = dev([root] if rank == 0 else [])
    dd, pp, vb = plc.bfs(h, Gb, srct, True, 0, True, False)
    bu = h.last_bfs_bottom_up_steps()
    mine = (v.cpu().numpy(), x.cpu().numpy(), it, vb.cpu().numpy(), dd.cpu().numpy(), pp.cpu().numpy(), bu)
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        vv = np.concatenate([a[0] for a in allr]).astype(np.int64)
        xx = np.concatenate([a[1] for a in allr])
        assert all(a[2] == it for a in allr)
        # single GPU, default numbering
        h1 = plc.ResourceHandle()
        G1 = plc.SGGraph(h1, props, dev(s), dev(d), None, store_transposed=True, renumber=True)
        v1, x1 = plc.pagerank(h1, G1, None, None, None, None, 0.85, 1e-6, 500, False)
        it1 = h1.last_iterations()
        v1, x1 = v1.cpu().numpy().astype(np.int64), x1.cpu().numpy()
        n = int(max(vv.max(), v1.max())) + 1
        a_mg, a_sg = np.zeros(n, np.float32), np.zeros(n, np.float32)
        a_mg[vv], a_sg[v1] = xx, x1
        print(f"RMAT-{scale} MG {world // C}x{C}: V={vv.size} E={E} PageRank iterations MG {it} SG {it1}, "
              f"equal bits {np.mean(a_mg[v1] == a_sg[v1]):.6f}; BFS bottom-up steps {[a[6] for a in allr]}")
        assert it == it1
        assert np.array_equal(a_mg.view(np.int32), a_sg.view(np.int32))
        G1 = None
        vb_all = np.concatenate([a[3] for a in allr]).astype(np.int64)  # MG global id order
        db_all = np.concatenate([a[4] for a in allr])
        pb_all = np.concatenate([a[5] for a in allr]).astype(np.int64)
        assert max(a[6] for a in allr) > 0  # the direction-optimising switch happened
        Gs = plc.SGGraph(h1, props, dev(s), dev(d), None, store_transposed=False, renumber=True)
        d1, _, u1 = plc.bfs(h1, Gs, dev([root]), True, 0, True, False)
        dist_sg = np.full(n, -7, np.int64)
        dist_sg[u1.cpu().numpy()] = d1.cpu().numpy()
        assert np.array_equal(db_all, dist_sg[vb_all])
        Gs = None
        inv = np.zeros(n, dtype=np.int64)
        inv[vb_all] = np.arange(vb_all.size)
        Gm = plc.SGGraph(h1, props, dev(inv[s]), dev(inv[d]), None, store_transposed=False, renumber=False)
        d2, p2, u2 = plc.bfs(h1, Gm, dev([inv[root]]), True, 0, True, False)
        assert np.array_equal(u2.cpu().numpy(), np.arange(vb_all.size))
        assert np.array_equal(d2.cpu().numpy(), db_all)
        pm = np.where(pb_all >= 0, inv[np.maximum(pb_all, 0)], -1)
        assert np.array_equal(p2.cpu().numpy().astype(np.int64), pm)
    dist.barrier()
    h = None
    Gb = None
    ctx.free()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,C,scale,chunks", [(8, 2, 18, None), (8, 8, 16, None), (2, 1, 16, None),
                                                  (8, 2, 16, 3), (4, 1, 14, 5)])
def test_mg_equals_sg(world, C, scale, chunks):
    """The reference's 8-GPU grid (4 x 2) at RMAT-18 and the flat 1 x 8 grid, rehearsed
    with 8 ranks on the one test GPU (torch.distributed/gloo callbacks).  chunks: the
    PageRank block's rows in that many chunks, pushed one after another with each
    chunk's column reduce-scatter on the comm stream (option mg_chunks; the default cuts
    4 chunks only from 64K rows per owner) -- still bitwise SG."""
    _spawn(_mg_sg_worker, (world, _free_port(), C, scale, chunks), world, deadline=300.0)


def _dask_worker(rank, world, port, C):
    """cugraph.dask (one process per GPU): each rank passes its partition of a raw
    edge list (duplicates, both directions, spread over the ranks) to
    Graph.from_dask_cudf_edgelist; PageRank / BFS / Louvain partitions, gathered, must
    match single-GPU cugraph on the whole edge list (the reference's
    python/cugraph/cugraph/tests/mg/test_mg_pagerank.py pattern):
    * PageRank bit for bit (u64 fixed-point sums and their u64 allreduce: the
      partition changes no sum; integer-valued weights keep the out-weight sums exact);
    * BFS distances exactly;
    * Louvain through one level -- MG and SG Louvain agree only through one level of
      the outer loop, and only on the same numbering (cpp/tests/community/
      mg_louvain_test.cpp:69-90,146-150): single-GPU Louvain with max_level 1 on the
      graph renumbered by the MG number map (the gathered result's vertex order) must
      give the same partition and the same modularity bits."""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _rank_setup(port, rank)
    import pandas as pd
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import cugraph
    from cugraph.dask.comms import comms as Comms
    from oracle import rmat

    s, d = rmat.rmat(10, 16 << 10, seed=9)
    w = (np.floor(rmat.rmat_weights(s.size, seed=10) * 8.0) + 1.0).astype(np.float32)
    df = pd.DataFrame({"src": s.astype(np.int64), "dst": d.astype(np.int64), "wt": w})
    Comms.initialize(pcols=C, backend="torch")
    assert Comms.get_2D_partition() == (world // C, C)
    part = df.iloc[rank::world]
    dg = cugraph.Graph(directed=False)
    dg.from_dask_cudf_edgelist(part, source="src", destination="dst", edge_attr="wt")
    pr = cugraph.dask.gather(cugraph.dask.pagerank(dg, tol=1e-6)).sort_values("vertex")
    root = int(s[0])
    bf = cugraph.dask.gather(cugraph.dask.bfs(dg, root)).sort_values("vertex")
    lv, q = cugraph.dask.louvain(dg, max_iter=1)
    lv = cugraph.dask.gather(lv)  # rank order: the MG global id order
    if rank == 0:
        g = cugraph.Graph(directed=False)
        g.from_pandas_edgelist(df, source="src", destination="dst", edge_attr="wt")
        ref = cugraph.pagerank(g, tol=1e-6).sort_values("vertex")
        assert np.array_equal(pr["vertex"].to_numpy(), ref["vertex"].to_numpy())
        assert np.array_equal(pr["pagerank"].to_numpy(), ref["pagerank"].to_numpy())
        rb = cugraph.bfs(g, root).sort_values("vertex")
        assert np.array_equal(bf["distance"].to_numpy(), rb["distance"].to_numpy())
        # Louvain: single-GPU Louvain, one level, on the MG-numbered graph
        import pylibcugraph as plc
        from oracle import graph as og
        nmap = lv["vertex"].to_numpy().astype(np.int64)
        assert np.array_equal(np.sort(nmap), ref["vertex"].to_numpy())
        inv = np.zeros(int(nmap.max()) + 1, dtype=np.int64)
        inv[nmap] = np.arange(nmap.size)
        ss, sd, sw = og.symmetrize_dedup(s.astype(np.int64), d.astype(np.int64), w.astype(np.float64))
        h1 = plc.ResourceHandle()
        G1 = plc.SGGraph(h1, plc.GraphProperties(is_symmetric=True, is_multigraph=False),
                         torch.as_tensor(inv[ss].astype(np.int32), device="cuda"),
                         torch.as_tensor(inv[sd].astype(np.int32), device="cuda"),
                         torch.as_tensor(sw.astype(np.float32), device="cuda"), store_transposed=False, renumber=False)
        v1, c1, q1 = plc.louvain(h1, G1, 1, 1.0, False)
        assert np.array_equal(v1.cpu().numpy(), np.arange(nmap.size))
        assert _same_partition(c1.cpu().numpy(), lv["partition"].to_numpy())
        assert q == q1, (q, q1)
    Comms.destroy()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,C", [(2, 1), (4, 2)])
def test_dask_api_vs_single_gpu(world, C):
    _spawn(_dask_worker, (world, _free_port(), C), world)


def _csr(V, src, dst, w):
    """CSR (offsets int64, indices int32, weights fp64) of a COO in ids [0, V), rows
    sorted by destination (the compiled oracle's input)."""
    order = np.lexsort((dst, src))
    off = np.zeros(V + 1, np.int64)
    np.cumsum(np.bincount(src, minlength=V), out=off[1:])
    return off, dst[order].astype(np.int32), w[order].astype(np.float64)


def _mg_rmat20_worker(rank, world, port, C, scale):
    """The reference's MG test size (RMAT(20, 32): mg_pagerank_test.cpp:333-347,
    mg_bfs_test.cpp:298, mg_louvain_test.cpp:270,307) on the reference's 8-GPU grid,
    rehearsed with 8 ranks on the one test GPU over gloo -- several ranks, so none of the
    one-rank shortcuts (the P == 1 contraction, the one-grid-row PageRank schedule) run.
    The graph is R-MAT(scale, 16) with integer weights 1..8, symmetrised, generated on
    the device by every rank (bit-identical to oracle/rmat.py).
    * PageRank (unweighted) bit for bit per external id against single-GPU PageRank,
      same iteration count;
    * BFS (direction-optimising) from the largest hub: distances equal to SG's,
      predecessors equal to SG's on the graph renumbered by the MG number map;
    * Louvain (integer weights: every sum exact): each MG dendrogram level is the
      compiled oracle's single-level Louvain (oracle/cpu_louvain.c, max_level 1) on the
      level graph numbered by the MG ids -- the same partition and the same modularity
      bits -- and the reported Q is the last improving level's
      (mg_louvain_test.cpp:82-151's method).  The graph has rows far over 1024 edges
      (the heavy-row passes k_big_*) and several levels (the P > 1 contraction's owner
      exchange)."""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    _rank_setup(port, rank)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pylibcugraph as plc

    h1 = plc.ResourceHandle()
    n = 16 << scale
    s, d = plc.generators.generate_rmat_edgelist(h1, scale, n, 0.57, 0.19, 0.19, 7, False, True)
    w = torch.floor(plc.generators.generate_edge_weights(h1, n, 8) * 8.0) + 1.0
    s, d, w = plc.generators.symmetrize_dedup(h1, s, d, w, True)
    E = s.numel()
    lo, hi = rank * E // world, (rank + 1) * E // world
    ctx = plc.comms.init_torch(C)
    h = plc.ResourceHandle(ctx.ptr)
    props = plc.GraphProperties(is_symmetric=True, is_multigraph=False)
    part = lambda t: t[lo:hi].contiguous()  # noqa: E731
    Gp = plc.MGGraph(h, props, part(s), part(d), None, store_transposed=True, num_edges=E)
    v, x = plc.pagerank(h, Gp, None, None, None, None, 0.85, 1e-6, 500, False)
    it = h.last_iterations()
    Gp = None
    Gb = plc.MGGraph(h, props, part(s), part(d), None, store_transposed=False, num_edges=E)
    deg = torch.bincount(s.to(torch.int64))
    root = int(torch.argmax(deg))
    maxdeg = int(deg.max())
    del deg
    dd, pp, vb = plc.bfs(h, Gb, torch.tensor([root] if rank == 0 else [], dtype=torch.int32, device="cuda"), True,
                         0, True, False)
    bu = h.last_bfs_bottom_up_steps()
    Gb = None
    Gl = plc.MGGraph(h, props, part(s), part(d), part(w), store_transposed=False, num_edges=E)
    lv_v, lv_c, q, levels = plc.louvain_dendrogram(h, Gl, 100, 1.0)
    Gl = None
    mine = (v.cpu().numpy(), x.cpu().numpy(), it, vb.cpu().numpy(), dd.cpu().numpy(), pp.cpu().numpy(), bu,
            lv_v.cpu().numpy(), lv_c.cpu().numpy(), q, [t.cpu().numpy() for t in levels])
    del v, x, vb, dd, pp, lv_v, lv_c, levels
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    if rank == 0:
        from oracle import cpu_native
        sh, dh, wh = s.cpu().numpy().astype(np.int64), d.cpu().numpy().astype(np.int64), w.cpu().numpy()
        # -- PageRank: bitwise SG
        vv = np.concatenate([a[0] for a in allr]).astype(np.int64)
        xx = np.concatenate([a[1] for a in allr])
        assert all(a[2] == it for a in allr)
        G1 = plc.SGGraph(h1, props, s, d, None, store_transposed=True, renumber=True)
        v1, x1 = plc.pagerank(h1, G1, None, None, None, None, 0.85, 1e-6, 500, False)
        it1 = h1.last_iterations()
        v1, x1 = v1.cpu().numpy().astype(np.int64), x1.cpu().numpy()
        G1 = None
        nx = int(max(vv.max(), v1.max())) + 1
        a_mg, a_sg = np.zeros(nx, np.float32), np.zeros(nx, np.float32)
        a_mg[vv], a_sg[v1] = xx, x1
        assert np.array_equal(np.sort(vv), np.sort(v1))
        print(f"RMAT-{scale} MG {world // C}x{C}: V={vv.size} E={E} max degree {maxdeg}; PageRank iterations MG {it} "
              f"SG {it1}, equal bits {np.mean(a_mg[v1] == a_sg[v1]):.6f}; BFS bottom-up steps {[a[6] for a in allr]}")
        assert it == it1
        assert np.array_equal(a_mg.view(np.int32), a_sg.view(np.int32)), "MG PageRank differs from SG"
        # -- BFS: distances = SG; predecessors = SG on the MG-numbered graph
        vb_all = np.concatenate([a[3] for a in allr]).astype(np.int64)
        db_all = np.concatenate([a[4] for a in allr])
        pb_all = np.concatenate([a[5] for a in allr]).astype(np.int64)
        assert max(a[6] for a in allr) > 0
        Gs = plc.SGGraph(h1, props, s, d, None, store_transposed=False, renumber=True)
        d1, _, u1 = plc.bfs(h1, Gs, torch.tensor([root], dtype=torch.int32, device="cuda"), True, 0, True, False)
        dist_sg = np.full(nx, -7, np.int64)
        dist_sg[u1.cpu().numpy()] = d1.cpu().numpy()
        Gs = None
        assert np.array_equal(db_all, dist_sg[vb_all]), "MG BFS distances differ from SG"
        inv = np.zeros(nx, dtype=np.int64)
        inv[vb_all] = np.arange(vb_all.size)
        dev = lambda a: torch.as_tensor(np.ascontiguousarray(a).astype(np.int32), device="cuda")  # noqa: E731
        Gm = plc.SGGraph(h1, props, dev(inv[sh]), dev(inv[dh]), None, store_transposed=False, renumber=False)
        d2, p2, u2 = plc.bfs(h1, Gm, dev([inv[root]]), True, 0, True, False)
        Gm = None
        assert np.array_equal(u2.cpu().numpy(), np.arange(vb_all.size))
        assert np.array_equal(d2.cpu().numpy(), db_all)
        pm = np.where(pb_all >= 0, inv[np.maximum(pb_all, 0)], -1)
        assert np.array_equal(p2.cpu().numpy().astype(np.int64), pm), "MG BFS predecessors differ from SG"
        # -- Louvain, level by level against the compiled oracle on the MG numbering
        nmap = np.concatenate([a[7] for a in allr]).astype(np.int64)
        assert np.array_equal(np.sort(nmap), np.sort(vb_all))
        inv = np.zeros(nx, dtype=np.int64)
        inv[nmap] = np.arange(nmap.size)
        L = len(allr[0][10])
        lv = [np.concatenate([a[10][i] for a in allr]).astype(np.int64) for i in range(L)]
        gs, gd, gw, V = inv[sh], inv[dh], wh.astype(np.float64), nmap.size
        best, qs = -1.0, []
        for i in range(L):
            assert lv[i].size == V
            off, idx, ww = _csr(V, gs, gd, gw)
            oc, oq, _ = cpu_native.louvain(off, idx, ww, max_level=1, threads=16)
            assert _same_partition(oc, lv[i]), f"level {i}: MG differs from the oracle's single level"
            qs.append(oq)
            if oq <= best:
                assert i == L - 1, "MG went on after a level without gain"
                break
            best = oq
            if i + 1 < L:  # coarsen by the MG level (mg_louvain_helper coarsen_graph)
                m = lv[i].max() + 1
                uk, inv_k = np.unique(lv[i][gs] * m + lv[i][gd], return_inverse=True)
                gw = np.bincount(inv_k, weights=gw)
                gs, gd = uk // m, uk % m
                V = lv[i + 1].size
        assert all(a[9] == q for a in allr)
        print(f"RMAT-{scale} MG Louvain {world} ranks: {L} levels, Q {q!r}, oracle per level {qs}")
        assert L >= 2, "a single level leaves the P > 1 contraction unexercised"
        assert q == best, (q, best)  # integer weights: the same bits
        flat = np.arange(nmap.size)
        for x_ in lv:
            flat = x_[flat]
        assert np.array_equal(np.concatenate([a[8] for a in allr]).astype(np.int64), flat)
    dist.barrier()
    h = None
    ctx.free()
    dist.destroy_process_group()


def test_mg_world8_rmat20_equals_sg():
    """8 ranks, the reference's 4 x 2 grid, RMAT-20 (see _mg_rmat20_worker)."""
    _spawn(_mg_rmat20_worker, (8, _free_port(), 2, 20), 8, deadline=600.0)

"""Parity at the benchmark sizes (the exact graphs bench.py builds and times).

* Graph structure of RMAT-22 and RMAT-24 (both orientations), checked
  independently of the library: the symmetrised, de-duplicated edge set is rebuilt
  from the same generator output with plain torch ops (sort + unique of
  ``min << 32 | max`` keys) and compared with the CSR/CSC edge set mapped through
  the number map; degrees are non-increasing in internal id with ties by ascending
  external id (create_graph_from_edgelist_impl.cuh:557-776,
  renumber_edgelist_impl.cuh:384-390, symmetrize.py:78-93); rows are strictly
  increasing (sorted, no multi-edges).
* PageRank on RMAT-22 (configs[1]), RMAT-24 (the headline) and RMAT-26 (the graph
  of configs[3], here on one GPU: V 32.8M, E 2.10G, the packed format's largest
  jump overhead and edge counts within 2.3 % of INT32_MAX): the HIP path
  against the fp64 oracle (oracle/cpu_baseline.c cpu_pagerank_f64 -- the numpy
  oracle's arithmetic compiled with OpenMP, checked against it in
  tests/test_cpu_baseline.py) at 1e-6 relative per vertex, same iteration count
  within one (the L1 sum order differs).  Unweighted (the C-ABI bench leg) and
  all-ones fp32 weights (what the reference's cugraph.Graph attaches,
  simpleGraph.py:840-843) on RMAT-22.
* BFS on RMAT-24 (configs[2]) from all 8 bench roots, direction-optimising:
  distances bit-exact against the compiled restatement of the reference's
  bfs_reference (bfs_test.cpp:41-79), plus Graph500-style full-size properties
  checked on the device (bfs_test.cpp:210-230 predecessor rule):
    d[src] = 0; no edge joins reached and unreached; |d[u] - d[v]| <= 1 on every
    edge; every reached v != src has a neighbour at d[v] - 1; and
    pred[v] = min{u in N(v) : d[u] = d[v] - 1} (the build's tie rule: smallest
    internal id), computed with scatter_reduce(amin).

Each bench graph is built once per module (fixtures) and shared by its tests.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

INF = 2**31 - 1
REL = 1e-6


def _bench():
    import bench
    import pylibcugraph as p
    return bench, p


def _cpu():
    from oracle import cpu_native
    cpu_native.lib()
    return cpu_native


class _Bench:
    """One bench graph (bench.build_rmat_graph) with its handle, number map and
    host copies of the adjacency, built once and shared by the module's tests."""

    def __init__(self, scale, want_roots=0):
        import torch
        bench, p = _bench()
        self.scale, self.p = scale, p
        self.h = p.ResourceHandle()
        self.g, self.roots, _ = bench.build_rmat_graph(p, self.h, scale, transposed=True, want_roots=want_roots)
        # result vertices are the number map in internal order (pagerank.cpp:231-237)
        v, _ = p.pagerank(self.h, self.g, None, None, None, None, 0.85, 1e-2, 500, False)
        self.number_map = v.to(torch.int64)
        self._host = {}

    def adjacency(self, transposed):
        return self.g.adjacency(self.h, transposed=transposed)

    def host_adjacency(self, transposed):
        if transposed not in self._host:
            off, idx, _ = self.adjacency(transposed)
            self._host[transposed] = (off.cpu().numpy().astype(np.int64), idx.cpu().numpy())
        return self._host[transposed]

    def close(self):
        import torch
        self.g = None
        self._host.clear()
        torch.cuda.synchronize()
        self.p.trim_device_cache()
        torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def rmat22():
    b = _Bench(22)
    yield b
    b.close()


@pytest.fixture(scope="module")
def rmat24():
    b = _Bench(24, want_roots=8)
    yield b
    b.close()


@pytest.fixture(scope="function")
def rmat26():  # (one test uses it: freed at once, before the RMAT-26 Louvain check)
    b = _Bench(26)
    yield b
    b.close()


def _check_structure(b, transposed):
    """The library's adjacency against an independent torch rebuild of the
    symmetrised, de-duplicated edge set of the same generator output."""
    import torch
    p, h = b.p, b.h
    n = 16 << b.scale
    s, d = p.generators.generate_rmat_edgelist(h, b.scale, n, 0.57, 0.19, 0.19, 42, False, True)
    s, d = s.to(torch.int64), d.to(torch.int64)
    lo, hi = torch.minimum(s, d), torch.maximum(s, d)
    del s, d
    want = torch.unique(lo << 32 | hi)  # sorted undirected edges, self loops once
    verts = torch.unique(torch.cat([lo, hi]))
    del lo, hi
    nm = b.number_map
    V = nm.numel()
    assert V == verts.numel(), "vertex count differs from the edge list's endpoint set"
    assert torch.equal(torch.sort(nm).values, verts), "number map is not the endpoint set"
    off, idx, w = b.adjacency(transposed)
    assert w is None
    off = off.to(torch.int64)
    assert off.numel() == V + 1 and int(off[0]) == 0
    deg = off[1:] - off[:-1]
    assert bool((deg[:-1] >= deg[1:]).all()), "degrees increase somewhere in internal id order"
    tie = deg[:-1] == deg[1:]
    assert bool((nm[:-1][tie] < nm[1:][tie]).all()), "equal-degree vertices not in ascending external id"
    rows = torch.repeat_interleave(torch.arange(V, device=off.device), deg)
    idx = idx.to(torch.int64)
    same_row = rows[1:] == rows[:-1]
    assert bool((idx[1:][same_row] > idx[:-1][same_row]).all()), "a row is unsorted or holds a multi-edge"
    u, v = nm[rows], nm[idx]
    del rows, idx, same_row
    if transposed:  # CSC: major = destination
        u, v = v, u
    fwd = u <= v
    got = torch.sort(u[fwd] << 32 | v[fwd]).values
    assert torch.equal(got, want), "edge set (u <= v) differs from the independent rebuild"
    back = torch.sort(v[~fwd] << 32 | u[~fwd]).values
    nonself = (want >> 32) != (want & 0xFFFFFFFF)
    assert torch.equal(back, want[nonself]), "the graph is not symmetric"
    E = u.numel()
    print(f"RMAT-{b.scale} {'CSC' if transposed else 'CSR'}: V={V} E={E} ({int(want.numel())} undirected) ok")
    assert E == b.g.number_of_edges()


@pytest.mark.parametrize("scale", [22, 24])
@pytest.mark.parametrize("transposed", [True, False])
def test_bench_graph_structure_independent(scale, transposed, request):
    _check_structure(request.getfixturevalue(f"rmat{scale}"), transposed)


def _pagerank_vs_oracle(b, g, weighted):
    import torch
    p, h = b.p, b.h
    v, pr = p.pagerank(h, g, None, None, None, None, 0.85, 1e-6, 500, False)
    it_gpu = h.last_iterations()
    assert torch.equal(v.to(torch.int64), b.number_map)
    off_h, idx_h = b.host_adjacency(True)
    ref, it_ref = _cpu().pagerank_f64(off_h, idx_h, 0.85, 1e-6, 500, threads=16)
    got = pr.cpu().numpy().astype(np.float64)
    rel = np.abs(got - ref) / ref
    print(f"RMAT-{b.scale}{' weighted' if weighted else ''}: V={ref.size} E={idx_h.size} iterations gpu {it_gpu} "
          f"oracle {it_ref} max rel {rel.max():.3e}")
    assert abs(it_gpu - it_ref) <= 1
    assert rel.max() < REL
    assert abs(got.sum() - 1.0) < 1e-4


@pytest.mark.parametrize("scale", [22, 24, 26])
def test_pagerank_bench_graph_vs_fp64_oracle(scale, request):
    b = request.getfixturevalue(f"rmat{scale}")
    _pagerank_vs_oracle(b, b.g, False)


def test_pagerank_rmat22_all_ones_weights_vs_fp64_oracle(rmat22):
    """The graph the reference's cugraph.Graph builds for an unweighted edge list:
    the same edges with all-ones fp32 weights (simpleGraph.py:840-843)."""
    import torch
    bench, p = _bench()
    b = rmat22
    g, _, _ = bench.build_rmat_graph(p, b.h, 22, transposed=True, weighted="ones")
    _pagerank_vs_oracle(b, g, True)
    del g
    torch.cuda.synchronize()


def _bfs_properties(off, idx, rows_all, dist, pred_ext, number_map, src, chunk=1 << 26):
    """Full-size device checks; off/idx the CSR (internal ids), rows_all the row of
    every CSR entry, dist by internal id, pred_ext external ids, number_map
    internal -> external."""
    import torch
    V = off.numel() - 1
    dev = dist.device
    d64 = dist.to(torch.int64)
    assert int(d64[src]) == 0
    minp = torch.full((V,), INF, dtype=torch.int64, device=dev)
    E = idx.numel()
    for lo in range(0, E, chunk):
        hi = min(E, lo + chunk)
        u = rows_all[lo:hi]
        v = idx[lo:hi].to(torch.int64)
        du, dv = d64[u], d64[v]
        ru, rv = du != INF, dv != INF
        assert bool((ru == rv).all()), "an edge joins the reached and unreached sets"
        both = ru & rv
        assert bool(((du - dv).abs()[both] <= 1).all()), "an edge spans more than one level"
        cand = both & (du == dv - 1)
        minp.scatter_reduce_(0, v[cand], u[cand], reduce="amin")
        del u, v, du, dv, ru, rv, both, cand
    reached = d64 != INF
    nonsrc = reached.clone()
    nonsrc[src] = False
    assert bool((minp[nonsrc] != INF).all()), "a reached vertex has no neighbour one level up"
    nm = number_map.to(torch.int64)
    want = torch.where(minp != INF, nm[minp.clamp(max=V - 1)], torch.full_like(minp, -1))
    want[src] = -1
    want[~reached] = -1
    assert bool((pred_ext.to(torch.int64) == want).all()), "predecessor is not the smallest-id parent"


def test_bfs_rmat24_all_bench_roots(rmat24):
    import torch
    b = rmat24
    p, h, g = b.p, b.h, b.g
    assert len(b.roots) == 8
    off, idx, _ = b.adjacency(False)
    off_h, idx_h = b.host_adjacency(False)
    deg = (off[1:] - off[:-1]).to(torch.int64)
    rows_all = torch.repeat_interleave(torch.arange(off.numel() - 1, device=off.device, dtype=torch.int64), deg)
    bottom_up = 0
    for r in b.roots:
        dist, pred, verts = p.bfs(h, g, torch.tensor([int(r)], dtype=torch.int32, device="cuda"), True, 0, True,
                                  False)
        bottom_up += h.last_bfs_bottom_up_steps()
        assert torch.equal(verts.to(torch.int64), b.number_map)
        src = int(torch.nonzero(b.number_map == int(r))[0, 0])
        _bfs_properties(off, idx, rows_all, dist, pred, verts, src)
        _, dref, _ = _cpu().bfs(off_h, idx_h, src, threads=16)
        assert np.array_equal(dist.cpu().numpy(), dref), f"root {r}: distances differ from the reference restatement"
        print(f"root {r}: reached {int((dref != INF).sum())}, levels {h.last_bfs_levels()}, "
              f"bottom-up steps {h.last_bfs_bottom_up_steps()}")
    assert bottom_up > 0  # the direction-optimising path was exercised
    del off, idx, rows_all, deg
    torch.cuda.synchronize()


def test_mg_one_rank_rccl_rmat24_equals_sg(rmat24):
    """The multi-GPU path at the headline size, through the library's RCCL
    communicators with the one rank a box allows: the MG graph build (its
    alltoallv moves 2.08 GB of edge ids: a single 2 GB ncclSend of a rank to
    itself once came back with a different graph), MG PageRank bit for bit equal to
    single-GPU PageRank (u64 fixed-point sums, u64 allreduce), MG BFS distances and
    predecessors equal to single-GPU BFS, by external id."""
    import os
    import torch
    import torch.distributed as dist
    bench, p = _bench()
    b = rmat24
    v, x = p.pagerank(b.h, b.g, None, None, None, None, 0.85, 1e-6, 500, False)
    it_sg = b.h.last_iterations()
    ext = v.to(torch.int64)
    n_ext = int(ext.max()) + 1
    sg_x = torch.zeros(n_ext, dtype=torch.int32, device="cuda")
    sg_x[ext] = x.view(torch.int32)
    root = int(b.roots[0])
    d, pr, vb = p.bfs(b.h, b.g, torch.tensor([root], dtype=torch.int32, device="cuda"), True, 0, True, False)
    sg_d = torch.full((n_ext,), -2, dtype=torch.int64, device="cuda")
    sg_p = torch.full((n_ext,), -2, dtype=torch.int64, device="cuda")
    sg_d[vb.to(torch.int64)] = d.to(torch.int64)
    sg_p[vb.to(torch.int64)] = pr.to(torch.int64)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(bench.free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    ctx = p.comms.init_rccl(1)
    try:
        hm = p.ResourceHandle(ctx.ptr)
        gm, _, _ = bench.build_rmat_graph(p, hm, 24, transposed=True, mg=(0, 1))
        assert gm.number_of_vertices() == b.g.number_of_vertices()
        assert gm.number_of_edges() == b.g.number_of_edges()
        vm, xm = p.pagerank(hm, gm, None, None, None, None, 0.85, 1e-6, 500, False)
        assert hm.last_iterations() == it_sg
        assert torch.equal(xm.view(torch.int32), sg_x[vm.to(torch.int64)]), "MG PageRank differs from SG"
        dm, pm, vmb = p.bfs(hm, gm, torch.tensor([root], dtype=torch.int32, device="cuda"), True, 0, True, False)
        ids = vmb.to(torch.int64)
        assert torch.equal(dm.to(torch.int64), sg_d[ids]), "MG BFS distances differ from SG"
        assert torch.equal(pm.to(torch.int64), sg_p[ids]), "MG BFS predecessors differ from SG"
        gm = None
        hm = None
        torch.cuda.synchronize()
        p.trim_device_cache()
    finally:
        ctx.free()
        dist.destroy_process_group()


class _OneRankRccl:
    """A torch.distributed world of one (gloo, for the unique-id broadcast) and the
    library's RCCL communicators over it: the MG code path with the one rank a box
    allows."""

    def __enter__(self):
        import os
        import torch.distributed as dist
        bench, p = _bench()
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ["MASTER_PORT"] = str(bench.free_port())
        dist.init_process_group("gloo", rank=0, world_size=1)
        self.ctx = p.comms.init_rccl(1)
        return self

    def __exit__(self, *exc):
        import torch
        import torch.distributed as dist
        _, p = _bench()
        torch.cuda.synchronize()
        p.trim_device_cache()
        self.ctx.free()
        dist.destroy_process_group()
        return False


def _by_ext(vertices, values, n_ext, fill=-2):
    """values scattered to external ids (int64 device tensor; `fill` where absent)."""
    import torch
    out = torch.full((n_ext,), fill, dtype=torch.int64, device=values.device)
    out[vertices.to(torch.int64)] = values.to(torch.int64)
    return out


def _free_device():
    """Return the library's and torch's cached device memory; (free, total) GB after."""
    import torch
    _, p = _bench()
    torch.cuda.synchronize()
    p.trim_device_cache()
    torch.cuda.empty_cache()
    f, t = torch.cuda.mem_get_info()
    return round(f / 2**30, 1), round(t / 2**30, 1)


def test_mg_one_rank_rccl_rmat26_equals_sg():
    """The multi-GPU path at the size of configs[3] and [4] (RMAT-26: V 32.8M, E 2.10G
    stored edges, 8.4 GB of edge ids through the MG build's alltoallv) through the
    library's RCCL communicators with one rank, against the single-GPU path on the same
    graph (the reference compares MG with SG at its RMAT use-case sizes,
    mg_pagerank_test.cpp:258-270, mg_louvain_test.cpp:40-46):
    * Louvain on the uniform [0, 1) fp32 weights of configs[4]: with one rank the MG
      algorithm is the SG one, so the clustering, the modularity's bits
      and the level count are identical;
    * PageRank bit for bit per external id, same iteration count;
    * BFS from the largest hub: distances and predecessors equal.
    Results are kept on the host between the phases: RMAT-26 Louvain's level graphs
    take > 100 GB of the device."""
    import time
    import torch
    bench, p = _bench()
    scale = 26
    n_ext = 1 << scale

    def timed(f):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = f()
        torch.cuda.synchronize()
        return r, time.perf_counter() - t0

    print("device memory free/total GB at start", _free_device())
    # -- single GPU: Louvain on the weighted graph
    h = p.ResourceHandle()
    g, _, _ = bench.build_rmat_graph(p, h, scale, weighted=True, transposed=False)
    p.louvain(h, g, 100, 1.0, False)  # (first call: allocator warm-up, as the MG call below is not)
    (v, c, q_sg), t_lv_sg = timed(lambda: p.louvain(h, g, 100, 1.0, False))
    lv_sg = h.last_louvain_levels()
    sg_c = _by_ext(v, c, n_ext).cpu()
    del v, c
    g = None
    _free_device()
    # -- single GPU: PageRank and BFS on the unweighted graph
    g, _, _ = bench.build_rmat_graph(p, h, scale, transposed=True)
    E = g.number_of_edges()
    v, x = p.pagerank(h, g, None, None, None, None, 0.85, 1e-6, 500, False)
    it_sg = h.last_iterations()
    _, t_pr_sg = timed(lambda: p.pagerank(h, g, None, None, None, None, 0.85, 1e-6, 500, False))  # steady call
    sg_x = _by_ext(v, x.view(torch.int32), n_ext).cpu()
    root = int(v[0])  # internal id 0: the largest degree
    d, pr, vb = p.bfs(h, g, torch.tensor([root], dtype=torch.int32, device="cuda"), True, 0, True, False)
    _, t_bfs_sg = timed(lambda: p.bfs(h, g, torch.tensor([root], dtype=torch.int32, device="cuda"), True, 0, True,
                                      False))
    sg_d, sg_p = _by_ext(vb, d, n_ext).cpu(), _by_ext(vb, pr, n_ext).cpu()
    del v, x, d, pr, vb
    g = None
    h = None
    print("device memory free/total GB after the SG phases", _free_device())
    # -- one-rank RCCL multi-GPU path
    with _OneRankRccl() as rc:
        hm = p.ResourceHandle(rc.ctx.ptr)
        gm, _, _ = bench.build_rmat_graph(p, hm, scale, weighted=True, transposed=False, mg=(0, 1))
        (vm, cm, q_mg), t_lv_mg = timed(lambda: p.louvain(hm, gm, 100, 1.0, False))
        assert hm.last_louvain_levels() == lv_sg
        assert q_mg == q_sg, (q_mg, q_sg)
        ids = vm.cpu().to(torch.int64)
        assert torch.equal(cm.cpu().to(torch.int64), sg_c[ids]), "MG Louvain clustering differs from SG at RMAT-26"
        del vm, cm, ids
        gm = None
        _free_device()
        gm, _, _ = bench.build_rmat_graph(p, hm, scale, transposed=True, mg=(0, 1))
        assert gm.number_of_edges() == E
        vm, xm = p.pagerank(hm, gm, None, None, None, None, 0.85, 1e-6, 500, False)
        assert hm.last_iterations() == it_sg
        assert torch.equal(xm.view(torch.int32).cpu().to(torch.int64), sg_x[vm.cpu().to(torch.int64)]), \
            "MG PageRank differs from SG at RMAT-26"
        _, t_pr_mg = timed(lambda: p.pagerank(hm, gm, None, None, None, None, 0.85, 1e-6, 500, False))
        dm, pm, vmb = p.bfs(hm, gm, torch.tensor([root], dtype=torch.int32, device="cuda"), True, 0, True, False)
        _, t_bfs_mg = timed(lambda: p.bfs(hm, gm, torch.tensor([root], dtype=torch.int32, device="cuda"), True, 0,
                                          True, False))
        ids = vmb.cpu().to(torch.int64)
        assert torch.equal(dm.cpu().to(torch.int64), sg_d[ids]), "MG BFS distances differ from SG at RMAT-26"
        assert torch.equal(pm.cpu().to(torch.int64), sg_p[ids]), "MG BFS predecessors differ from SG at RMAT-26"
        print(f"RMAT-26 one-rank RCCL MG == SG: PageRank {it_sg} iterations, BFS from {root}, "
              f"Louvain Q {q_sg:.9f} in {lv_sg} levels")
        # the one-rank MG path's cost over SG (steady PageRank and BFS calls; Louvain end
        # to end, the SG time from its second call)
        print(f"RMAT-26 MG/SG time: PageRank {t_pr_mg / t_pr_sg:.3f} ({1e3 * t_pr_mg:.2f} / {1e3 * t_pr_sg:.2f} ms), "
              f"BFS {t_bfs_mg / t_bfs_sg:.3f} ({1e3 * t_bfs_mg:.2f} / {1e3 * t_bfs_sg:.2f} ms), "
              f"Louvain {t_lv_mg / t_lv_sg:.3f} ({t_lv_mg:.2f} / {t_lv_sg:.2f} s)")
        del vm, xm, dm, pm, vmb
        gm = None
        hm = None
    _free_device()


def test_mg_one_rank_rccl_louvain_rmat20_integer_equals_sg():
    """Integer weights (every sum exact on either path): one-rank RCCL MG Louvain on
    RMAT-20 gives SG's clustering, modularity bits and level count."""
    import torch
    bench, p = _bench()
    h = p.ResourceHandle()
    n = 16 << 20
    s, d = p.generators.generate_rmat_edgelist(h, 20, n, 0.57, 0.19, 0.19, 7, False, True)
    w = torch.floor(p.generators.generate_edge_weights(h, n, 8) * 8.0) + 1.0
    s, d, w = p.generators.symmetrize_dedup(h, s, d, w, True)
    props = p.GraphProperties(is_symmetric=True, is_multigraph=False)
    g = p.SGGraph(h, props, s, d, w, store_transposed=False, renumber=True)
    v, c, q_sg = p.louvain(h, g, 100, 1.0, False)
    lv_sg = h.last_louvain_levels()
    sg_c = _by_ext(v, c, 1 << 20)
    g = None
    with _OneRankRccl() as rc:
        hm = p.ResourceHandle(rc.ctx.ptr)
        gm = p.MGGraph(hm, props, s, d, w, store_transposed=False, num_edges=s.numel())
        vm, cm, q_mg = p.louvain(hm, gm, 100, 1.0, False)
        assert hm.last_louvain_levels() == lv_sg and q_mg == q_sg, (q_mg, q_sg)
        assert torch.equal(cm.to(torch.int64), sg_c[vm.to(torch.int64)])
        gm = None
        hm = None


def _louvain_q_recomputed(scale):
    """Louvain on a bench graph (symmetric R-MAT, fp32 [0,1) weights, bench.py
    louvain_leg): the reported Q is the modularity of the returned partition,
    recomputed on the device in fp64 from the library's own adjacency
    (compute_modularity, common_methods.cuh:121-170): internal weight / m -
    sum_c a_c^2 / m^2, over edge chunks."""
    import torch
    bench, p = _bench()
    h = p.ResourceHandle()
    g, _, _ = bench.build_rmat_graph(p, h, scale, weighted=True, transposed=False)
    v, c, q = p.louvain(h, g, 100, 1.0, False)
    levels = h.last_louvain_levels()
    del v
    off, idx, w = g.adjacency(h, transposed=False)
    g = None
    p.trim_device_cache()  # Louvain's level graphs (RMAT-26: > 100 GB) go back to the device
    torch.cuda.empty_cache()
    V = off.numel() - 1
    c = c.to(torch.int64)
    off64 = off.to(torch.int64)
    del off
    E = idx.numel()
    internal = torch.zeros((), dtype=torch.float64, device=idx.device)
    chunk = 1 << 28
    for lo in range(0, E, chunk):
        hi = min(E, lo + chunk)
        # rows of edges [lo, hi): searchsorted on the offsets (no E-sized row array)
        rows = torch.searchsorted(off64, torch.arange(lo, hi, device=idx.device, dtype=torch.int64), right=True) - 1
        wc = w[lo:hi].to(torch.float64)
        internal += torch.where(c[rows] == c[idx[lo:hi].to(torch.int64)], wc, torch.zeros_like(wc)).sum()
        del rows, wc
    # vertex weights k from a prefix sum of 2^32 fixed-point weights (exact integer
    # differences; an index_add_ of E fp64 atomics onto the hub rows took minutes and a
    # fp64 prefix sum loses the small rows' bits to cancellation)
    cs = torch.zeros(E + 1, dtype=torch.int64, device=idx.device)
    carry = 0
    for lo in range(0, E, chunk):
        hi = min(E, lo + chunk)
        part = torch.cumsum(torch.round(w[lo:hi].to(torch.float64) * 2.0**32).to(torch.int64), 0)
        cs[lo + 1:hi + 1] = part + carry
        carry = int(part[-1]) + carry
        del part
    kf = cs[off64[1:]] - cs[off64[:-1]]  # vertex weights, 2^32 fixed point
    m = cs[-1].to(torch.float64) * 2.0**-32
    del cs
    # cluster weights: sort by cluster and segment-sum the fixed-point k (an index_add_
    # of every vertex onto the few large final clusters serialises on their addresses)
    cv, order = torch.sort(c)
    ck = torch.cumsum(kf[order], 0)
    ends = torch.cat([torch.nonzero(cv[1:] != cv[:-1]).flatten(), torch.tensor([V - 1], device=cv.device)])
    tot = ck[ends]
    a = torch.cat([tot[:1], tot[1:] - tot[:-1]]).to(torch.float64) * 2.0**-32
    del cv, order, ck, ends, tot, kf
    Q = float(internal / m - (a * a).sum() / (m * m))
    print(f"RMAT-{scale} Louvain: V={V} E={E} Q reported {q:.12f} recomputed {Q:.12f}, levels {levels}, "
          f"clusters {int(torch.unique(c).numel())}")
    del off64, idx, w, c, a
    torch.cuda.synchronize()
    p.trim_device_cache()
    torch.cuda.empty_cache()
    return q, Q


@pytest.mark.parametrize("scale", [23, 26])
def test_louvain_bench_graph_modularity(scale):
    """RMAT-23 (bench.py's N=1 Louvain leg) and RMAT-26 (the graph of configs[4], here
    on one GPU): reported Q == recomputed Q to 1e-9 relative."""
    q, Q = _louvain_q_recomputed(scale)
    assert abs(Q - q) <= 1e-9 * abs(q)
    assert q > 0.05


def test_louvain_hash_equals_sort_rmat20():
    """RMAT-20 with integer weights: the LDS-hash local move (multi-segment heavy
    rows, many buckets per row) and the sort local move give the same clustering."""
    import torch
    bench, p = _bench()
    h = p.ResourceHandle()
    n = 16 << 20
    s, d = p.generators.generate_rmat_edgelist(h, 20, n, 0.57, 0.19, 0.19, 7, False, True)
    w = torch.floor(p.generators.generate_edge_weights(h, n, 8) * 8.0) + 1.0
    s, d, w = p.generators.symmetrize_dedup(h, s, d, w, True)
    props = p.GraphProperties(is_symmetric=True, is_multigraph=False)
    out = []
    for mode in (1, 0):
        h.set_option("louvain_hash", mode)
        g = p.SGGraph(h, props, s, d, w, store_transposed=False, renumber=True)
        v, c, q = p.louvain(h, g, 100, 1.0, False)
        out.append((v.cpu().numpy(), c.cpu().numpy(), q, h.last_louvain_levels()))
        del g
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2] and out[0][3] == out[1][3]

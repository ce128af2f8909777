"""Parity at the benchmark sizes (the exact graphs bench.py builds and times).

* PageRank on RMAT-22 (configs[1]) and RMAT-24 (the headline): the HIP path
  against the fp64 oracle (oracle/cpu_baseline.c cpu_pagerank_f64 -- the numpy
  oracle's arithmetic compiled with OpenMP, checked against it in
  tests/test_cpu_baseline.py) at 1e-6 relative per vertex, same iteration count
  within one (the L1 sum order differs).
* BFS on RMAT-24 (configs[2]) from all 8 bench roots, direction-optimising:
  distances bit-exact against the compiled restatement of the reference's
  bfs_reference (bfs_test.cpp:41-79), plus Graph500-style full-size properties
  checked on the device (bfs_test.cpp:210-230 predecessor rule):
    d[src] = 0; no edge joins reached and unreached; |d[u] - d[v]| <= 1 on every
    edge; every reached v != src has a neighbour at d[v] - 1; and
    pred[v] = min{u in N(v) : d[u] = d[v] - 1} (the build's tie rule: smallest
    internal id), computed with scatter_reduce(amin).

The oracle input is the library's own adjacency of the GPU-built graph (graph
construction is pinned against the oracle's at smaller scales by
tests/test_gpu_rmat.py and the dataset tests).
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


@pytest.mark.parametrize("scale", [22, 24])
def test_pagerank_bench_graph_vs_fp64_oracle(scale):
    import torch
    bench, p = _bench()
    cpu = _cpu()
    h = p.ResourceHandle()
    g, _, _ = bench.build_rmat_graph(p, h, scale, transposed=True)
    v, pr = p.pagerank(h, g, None, None, None, None, 0.85, 1e-6, 500, False)
    it_gpu = h.last_iterations()
    off, idx, _ = g.adjacency(h, transposed=True)
    off_h, idx_h = off.cpu().numpy().astype(np.int64), idx.cpu().numpy()
    del off, idx
    ref, it_ref = cpu.pagerank_f64(off_h, idx_h, 0.85, 1e-6, 500, threads=16)
    got = pr.cpu().numpy().astype(np.float64)
    rel = np.abs(got - ref) / ref
    print(f"RMAT-{scale}: V={ref.size} E={idx_h.size} iterations gpu {it_gpu} oracle {it_ref} "
          f"max rel {rel.max():.3e}")
    assert abs(it_gpu - it_ref) <= 1
    assert rel.max() < REL
    assert abs(got.sum() - 1.0) < 1e-4
    del g
    torch.cuda.synchronize()
    p.trim_device_cache()


def _bfs_properties(off, idx, dist, pred_ext, number_map, src, chunk=1 << 26):
    """Full-size device checks; off/idx the CSR (internal ids), dist by internal id,
    pred_ext external ids, number_map internal -> external."""
    import torch
    V = off.numel() - 1
    dev = dist.device
    d64 = dist.to(torch.int64)
    assert int(d64[src]) == 0
    minp = torch.full((V,), INF, dtype=torch.int64, device=dev)
    deg = (off[1:] - off[:-1]).to(torch.int64)
    rows_all = torch.repeat_interleave(torch.arange(V, device=dev, dtype=torch.int64), deg)
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
    del rows_all
    reached = d64 != INF
    nonsrc = reached.clone()
    nonsrc[src] = False
    assert bool((minp[nonsrc] != INF).all()), "a reached vertex has no neighbour one level up"
    nm = number_map.to(torch.int64)
    want = torch.where(minp != INF, nm[minp.clamp(max=V - 1)], torch.full_like(minp, -1))
    want[src] = -1
    want[~reached] = -1
    assert bool((pred_ext.to(torch.int64) == want).all()), "predecessor is not the smallest-id parent"


def test_bfs_rmat24_all_bench_roots():
    import torch
    bench, p = _bench()
    cpu = _cpu()
    h = p.ResourceHandle()
    g, roots, _ = bench.build_rmat_graph(p, h, 24, transposed=False, want_roots=8)
    assert len(roots) == 8
    off, idx, _ = g.adjacency(h, transposed=False)
    off_h, idx_h = off.cpu().numpy().astype(np.int64), idx.cpu().numpy()
    bottom_up = 0
    for r in roots:
        dist, pred, verts = p.bfs(h, g, torch.tensor([int(r)], dtype=torch.int32, device="cuda"), True, 0, True,
                                  False)
        bottom_up += h.last_bfs_bottom_up_steps()
        vh = verts.cpu().numpy()
        src = int(np.nonzero(vh == r)[0][0])
        _bfs_properties(off, idx, dist, pred, verts, src)
        _, dref, _ = cpu.bfs(off_h, idx_h, src, threads=16)
        assert np.array_equal(dist.cpu().numpy(), dref), f"root {r}: distances differ from the reference restatement"
        print(f"root {r}: reached {int((dref != INF).sum())}, levels {h.last_bfs_levels()}, "
              f"bottom-up steps {h.last_bfs_bottom_up_steps()}")
    assert bottom_up > 0  # the direction-optimising path was exercised
    del g, off, idx
    torch.cuda.synchronize()
    p.trim_device_cache()


def test_louvain_bench_graph_modularity():
    """Louvain on the bench graph (RMAT-23, fp32 [0,1) weights, bench.py louvain_leg):
    the reported Q is the modularity of the returned partition, recomputed on the
    device in fp64 from the library's own adjacency (compute_modularity,
    common_methods.cuh:121-170): internal weight / m - sum_c a_c^2 / m^2."""
    import torch
    bench, p = _bench()
    h = p.ResourceHandle()
    g, _, _ = bench.build_rmat_graph(p, h, 23, weighted=True, transposed=False)
    v, c, q = p.louvain(h, g, 100, 1.0, False)
    off, idx, w = g.adjacency(h, transposed=False)
    V = off.numel() - 1
    c = c.to(torch.int64)
    deg = (off[1:] - off[:-1]).to(torch.int64)
    rows = torch.repeat_interleave(torch.arange(V, device=off.device), deg)
    w64 = w.to(torch.float64)
    m = w64.sum()
    internal = torch.where(c[rows] == c[idx.to(torch.int64)], w64, torch.zeros_like(w64)).sum()
    k = torch.zeros(V, dtype=torch.float64, device=off.device).index_add_(0, rows, w64)
    a = torch.zeros(int(c.max()) + 1, dtype=torch.float64, device=off.device).index_add_(0, c, k)
    Q = float(internal / m - (a * a).sum() / (m * m))
    print(f"RMAT-23 Louvain: Q reported {q:.12f} recomputed {Q:.12f}, levels {h.last_louvain_levels()}, "
          f"clusters {int(torch.unique(c).numel())}")
    assert abs(Q - q) <= 1e-9 * abs(q)
    assert q > 0.05
    del g, off, idx, w, rows, w64
    torch.cuda.synchronize()
    p.trim_device_cache()


def test_louvain_hash_equals_sort_rmat20(monkeypatch):
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
    for mode in ("1", "0"):
        monkeypatch.setenv("CGX_LOUVAIN_HASH", mode)
        g = p.SGGraph(h, props, s, d, w, store_transposed=False, renumber=True)
        v, c, q = p.louvain(h, g, 100, 1.0, False)
        out.append((v.cpu().numpy(), c.cpu().numpy(), q, h.last_louvain_levels()))
        del g
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2] and out[0][3] == out[1][3]

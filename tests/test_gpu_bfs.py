"""BFS parity: distances bit-exact vs the oracle; predecessors exact under the
documented tie rule (smallest internal id), and valid per bfs_test.cpp:210-230."""
import numpy as np
import pytest

from conftest import dataset_path
from gpu_util import host, make_graph, plc
from oracle import bfs as obfs
from oracle import graph as og
from oracle import rmat

pytestmark = pytest.mark.gpu
INT32_MAX = 2**31 - 1


def run(h, G, sources, do, depth=0, pred=True, vdtype=np.int32):
    d, p, v = plc().bfs(h, G, np.asarray(sources, vdtype), do, depth, pred, False)
    return host(v), host(d), host(p)


def check_vs_oracle(s, d, v, dist, pred, sources_ext, depth_limit=None, inf=INT32_MAX):
    n_ext = int(max(np.max(s, initial=0), np.max(d, initial=0), np.max(sources_ext))) + 1
    G = og.create_graph(s, d, None, renumber=False, vertices=np.arange(n_ext))
    key = np.full(n_ext, np.iinfo(np.int64).max // 2, dtype=np.int64)
    key[v] = np.arange(v.size)  # internal id = position in the result arrays
    # make the key a permutation (ids absent from the GPU graph never win)
    absent = np.setdiff1d(np.arange(n_ext), v)
    key[absent] = v.size + np.arange(absent.size)
    rd, rp = obfs.bfs(n_ext, G.offsets, G.indices, sources_ext, depth_limit, tie_key=key, invalid_distance=inf)
    assert np.array_equal(dist, rd[v])
    if pred is not None and pred.size:
        assert np.array_equal(pred, rp[v])


def test_c_golden(golden):
    g = golden["bfs_c"]
    for transposed in (False, True):
        h, G = make_graph(g["src"], g["dst"], g["w"], transposed=transposed, renumber=False)
        v, dist, pred = run(h, G, g["sources"], False, g["depth_limit"])
        exp_d = np.asarray(g["expected_distances"])
        exp_p = np.asarray(g["expected_predecessors"])
        assert np.array_equal(dist, exp_d[v]) and np.array_equal(pred, exp_p[v])


@pytest.mark.parametrize("name", ["karate.csv", "dolphins.csv", "netscience.csv"])
@pytest.mark.parametrize("do", [False, True])
def test_datasets(name, do):
    s, d, _ = og.read_csv(dataset_path(name))
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    src = [int(s[0])]
    v, dist, pred = run(h, G, src, do)
    check_vs_oracle(s, d, v, dist, pred, src)


def rmat_sym(scale, seed=42):
    s, d = rmat.rmat(scale, 16 << scale, seed=seed)
    s, d, _ = og.symmetrize_dedup(s, d)
    return s, d


@pytest.mark.parametrize("scale", [10, 14])
@pytest.mark.parametrize("do", [False, True])
def test_rmat(scale, do):
    s, d = rmat_sym(scale)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    deg = np.bincount(s)
    src = [int(np.argmax(deg))]
    v, dist, pred = run(h, G, src, do)
    check_vs_oracle(s, d, v, dist, pred, src)
    if do and scale == 14:
        assert h.last_bfs_bottom_up_steps() > 0  # the bottom-up path was exercised


def test_rmat_multi_source_and_depth_limit():
    s, d = rmat_sym(12)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    verts = np.unique(s)
    srcs = [int(verts[3]), int(verts[100]), int(verts[100]), int(verts[-1])]
    for do in (False, True):
        v, dist, pred = run(h, G, srcs, do, depth=2)
        check_vs_oracle(s, d, v, dist, pred, srcs, depth_limit=2)
        assert dist[dist != INT32_MAX].max() <= 2


def test_directed_top_down_and_do_requires_symmetric():
    s, d = rmat.rmat(11, 16 << 11)
    s, d, _ = og.symmetrize_dedup(s, d, symmetrize=False)
    h, G = make_graph(s, d, None, renumber=True, symmetric=False)
    src = [int(s[0])]
    v, dist, pred = run(h, G, src, False)
    check_vs_oracle(s, d, v, dist, pred, src)
    with pytest.raises(ValueError, match="symmetric"):
        run(h, G, src, True)


def test_int64_no_predecessors():
    s, d = rmat_sym(11)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True, vdtype=np.int64)
    v, dist, pred = run(h, G, [int(s[0])], True, pred=False, vdtype=np.int64)
    assert pred.size == 0
    check_vs_oracle(s, d, v, dist, None, [int(s[0])], inf=np.iinfo(np.int64).max)


def test_invalid_source():
    h, G = make_graph([0, 1], [1, 2], None, renumber=True)
    with pytest.raises(ValueError):
        run(h, G, [7], False)


def test_isolated_source_and_unrenumbered_gaps():
    # ids 0..9 with vertex 5 isolated (renumber=False keeps it)
    h, G = make_graph([0, 1, 2, 6], [1, 2, 3, 7], None, renumber=False, symmetric=False)
    v, dist, pred = run(h, G, [5], False)
    assert dist[v == 5][0] == 0 and np.all(dist[v != 5] == INT32_MAX)


@pytest.mark.parametrize("scale", [12, 16])
def test_unrenumbered_direction_optimising(scale):
    """renumber=False with ids that do not descend by degree: the bottom-up levels run
    the one-pass k_bottomup over the degree-binned work items (not the probe, which
    needs the identity order), predecessors stay internal = external ids.  Same
    arrays as the top-down-only traversal, and the oracle at 12."""
    s, d = rmat_sym(scale)
    n = int(max(s.max(), d.max())) + 1
    perm = np.random.default_rng(3).permutation(n)
    ps, pd_ = perm[s], perm[d]
    h, G = make_graph(ps, pd_, None, renumber=False, symmetric=True)
    deg = np.bincount(ps, minlength=n)
    for x in (int(np.argmax(deg)), int(ps[len(ps) // 2])):
        v0, d0, p0 = run(h, G, [x], False)
        v, dist, pred = run(h, G, [x], True)
        assert h.last_bfs_bottom_up_steps() > 0
        assert np.array_equal(v, v0) and np.array_equal(dist, d0) and np.array_equal(pred, p0)
        if scale == 12:
            check_vs_oracle(ps, pd_, v, dist, pred, [x])


@pytest.mark.parametrize("transposed", [False, True])
def test_extract_paths_c_golden(golden, transposed):
    g = golden["extract_paths_c"]
    h, G = make_graph(g["src"], g["dst"], g["w"], transposed=transposed, renumber=False)
    paths, L = plc().bfs_paths(h, G, np.asarray(g["sources"], np.int32), np.asarray(g["destinations"], np.int32),
                               g["depth_limit"])
    assert L == g["expected_max_path_length"]
    assert host(paths).ravel().tolist() == g["expected_paths"]


def test_extract_paths_rmat_renumbered():
    """Every extracted path starts at the source, follows edges, ends at its destination
    and has distance + 1 vertices; unreachable destinations give an all -1 row."""
    s, d = rmat.rmat(10, 16 << 10, seed=3)
    s, d, _ = og.symmetrize_dedup(s, d)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    root = int(s[0])
    dests = np.unique(np.concatenate([s[:50], d[:50]])).astype(np.int32)
    paths, L = plc().bfs_paths(h, G, np.asarray([root], np.int32), dests)
    dist, _, verts = plc().bfs(h, G, np.asarray([root], np.int32), False, 0, True, False)
    dmap = dict(zip(host(verts).tolist(), host(dist).tolist()))
    P = host(paths)
    edges = set(zip(s.tolist(), d.tolist()))
    assert L == 1 + max(dmap[int(x)] for x in dests if dmap[int(x)] < 2**31 - 1)
    for row, dv in zip(P, dests):
        seq = [int(x) for x in row if x != -1]
        if dmap[int(dv)] == 2**31 - 1:
            assert seq == []
            continue
        assert seq[0] == root and seq[-1] == dv and len(seq) == dmap[int(dv)] + 1
        assert all((a, b) in edges for a, b in zip(seq, seq[1:]))


@pytest.mark.parametrize("scale", [14, 18])
def test_probe_vector_loads_same_result(scale):
    """Every bottom-up probe form gives the same distances and predecessors: the
    default (bfs.hip k_bu_probe<HEAD, STAGE2>: the 16-byte head table's first 3
    neighbours, then neighbours 3..10 by 16-byte loads of the padded adjacency), the
    head table alone (option bfs_probe_vec = 0, which also turns off the vector loads), and
    the adjacency probe without the head table (bfs_head = 0: 8 neighbours by
    16-byte loads)."""
    s, d = rmat_sym(scale)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    deg = np.bincount(s)
    srcs = [int(np.argmax(deg)), int(s[len(s) // 3]), int(d[-1])]
    h.set_option("bfs_probe_vec", 0)
    base = [run(h, G, [x], True) for x in srcs]
    h.set_option("bfs_probe_vec", 1)
    h.set_option("bfs_head", 0)
    nohead = [run(h, G, [x], True) for x in srcs]
    h.set_option("bfs_head", 1)
    for (v0, d0, p0), (v1, d1, p1) in zip(base, nohead):
        assert np.array_equal(v1, v0) and np.array_equal(d1, d0) and np.array_equal(p1, p0)
    for x, (v0, d0, p0) in zip(srcs, base):
        v, dist, pred = run(h, G, [x], True)
        assert h.last_bfs_bottom_up_steps() > 0
        assert np.array_equal(v, v0) and np.array_equal(dist, d0) and np.array_equal(pred, p0)
        if scale == 14:
            check_vs_oracle(s, d, v, dist, pred, [x])


@pytest.mark.parametrize("scale", [14, 18])
def test_predecessors_every_level_kind(scale):
    """External-id predecessors are written during the traversal: bottom-up levels
    store them directly, a top-down level's (smallest parent by atomicMin on internal
    ids) are translated when its queue is marked -- or after the loop when a depth
    limit ends it.  Direction-optimising and top-down-only traversals (which take
    different paths through that) must give the same arrays, with and without a
    depth limit, from one and several sources; checked against the oracle at 14."""
    s, d = rmat_sym(scale)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    deg = np.bincount(s)
    cases = [([int(np.argmax(deg))], 0), ([int(s[len(s) // 3])], 0), ([int(d[-1])], 0),
             ([int(s[7]), int(d[11])], 2), ([int(s[5])], 3), ([int(s[9])], 1)]
    for x, depth in cases:
        v0, d0, p0 = run(h, G, x, False, depth)
        v, dist, pred = run(h, G, x, True, depth)
        assert np.array_equal(v, v0) and np.array_equal(dist, d0) and np.array_equal(pred, p0), (x, depth)
        if scale == 14:
            check_vs_oracle(s, d, v, dist, pred, x, depth_limit=depth or None)


def test_result_tensors_own_library_memory():
    """Result tensors view the library's result arrays without a copy
    (pylibcugraph._arrays.views_to_tensors_owned): they must stay intact across
    later calls (which allocate from the same cache) and after a derived tensor
    outlives the original ones."""
    import gc
    s, d = rmat_sym(12)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    dist, pred, verts = plc().bfs(h, G, np.asarray([int(s[0])], np.int32), True, 0, True, False)
    snap = (host(dist).copy(), host(pred).copy(), host(verts).copy())
    view = dist[1:]  # shares the storage
    del dist
    gc.collect()
    for x in (int(s[5]), int(d[7]), int(s[-1])):
        plc().bfs(h, G, np.asarray([x], np.int32), True, 0, True, False)
        plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 100, False)
    gc.collect()
    assert np.array_equal(host(view), snap[0][1:])
    assert np.array_equal(host(pred), snap[1]) and np.array_equal(host(verts), snap[2])


@pytest.mark.parametrize("scale", [14, 18])
def test_bitmap_to_queue_conversion_device_vs_host(scale, monkeypatch, capfd):
    """A bottom-up -> top-down switch converts the frontier bitmap to queues with the
    queue lengths read on the device: same distances and predecessors as the
    top-down-only traversal (which converts nothing), and the runs do contain such a
    switch (CGX_BFS_DEBUG level log)."""
    s, d = rmat_sym(scale)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    deg = np.bincount(s)
    srcs = [int(np.argmax(deg)), int(s[len(s) // 3])]
    monkeypatch.setenv("CGX_BFS_DEBUG", "1")
    capfd.readouterr()
    base = [run(h, G, [x], True) for x in srcs]
    log = capfd.readouterr().err
    dirs = [ln.split()[3] for ln in log.splitlines() if ln.startswith("[bfs] level")]
    assert any(a == "bottom-up" and b == "top-down" for a, b in zip(dirs, dirs[1:])), log[-2000:]
    for x, (v0, d0, p0) in zip(srcs, base):
        v, dist, pred = run(h, G, [x], False)
        assert np.array_equal(v, v0) and np.array_equal(dist, d0) and np.array_equal(pred, p0)
    if scale == 14:
        for x, (v0, d0, p0) in zip(srcs, base):
            check_vs_oracle(s, d, v0, d0, p0, [x])


def test_result_freed_after_side_stream_reader():
    """A result tensor read on a non-default stream, then dropped: its memory goes
    back to the library's cache only after the device is synchronised
    (ResultOwner.__del__), so the next algorithm's arrays cannot overwrite it while
    the side-stream reader still runs."""
    import gc
    import torch
    s, d = rmat_sym(16)
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    src = np.asarray([int(s[0])], np.int32)
    dist, pred, verts = plc().bfs(h, G, src, True, 0, True, False)
    want = dist.clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        acc = torch.zeros_like(dist, dtype=torch.int64)
        for _ in range(50):  # a long reader queued on the side stream
            acc += dist.to(torch.int64)
    del dist, pred, verts
    gc.collect()
    plc().bfs(h, G, np.asarray([int(d[-1])], np.int32), True, 0, True, False)
    torch.cuda.synchronize()
    assert torch.equal(acc, want.to(torch.int64) * 50)

"""PageRank parity: HIP path (through the C ABI) vs the oracle and the reference's
golden vectors.  Tolerance: 1e-6 relative vs the fp64 oracle (north_star)."""
import functools

import numpy as np
import pytest

from conftest import dataset_path
from gpu_util import host, make_graph, plc
from oracle import graph as og
from oracle import pagerank as opr
from oracle import rmat

pytestmark = pytest.mark.gpu

REL = 1e-6


def by_ext(vertices, values):
    v, x = host(vertices), host(values)
    out = np.zeros(v.max() + 1 if v.size else 0, dtype=np.float64)
    out[v] = x
    return out


@pytest.mark.parametrize("case", ["pagerank_c_6v", "pagerank_c_4path"])
@pytest.mark.parametrize("transposed", [True, False])
def test_c_golden(golden, case, transposed):
    g = golden[case]
    h, G = make_graph(g["src"], g["dst"], g["w"], transposed=transposed, renumber=False)
    v, pr = plc().pagerank(h, G, None, None, None, None, g["alpha"], g["epsilon"], g["max_iterations"], False)
    got = by_ext(v, pr)
    exp = np.asarray(g["expected"])
    assert np.all(np.abs(got - exp) <= g["tol"] * np.maximum(np.abs(got), np.abs(exp)))
    ref = opr.pagerank(g["num_vertices"], g["src"], g["dst"], np.asarray(g["w"], np.float32).astype(np.float64),
                       g["alpha"], g["epsilon"], g["max_iterations"])
    assert np.max(np.abs(got - ref) / ref) < REL


def test_c_golden_personalized(golden):
    g = golden["pagerank_c_personalized"]
    h, G = make_graph(g["src"], g["dst"], g["w"], transposed=True, renumber=False)
    v, pr = plc().personalized_pagerank(h, G, None, None, None, None,
                                        np.asarray(g["personalization_vertices"], np.int32),
                                        np.asarray(g["personalization_values"], np.float32),
                                        g["alpha"], g["epsilon"], g["max_iterations"], False)
    got = by_ext(v, pr)
    exp = np.asarray(g["expected"])
    assert np.all(np.abs(got - exp) <= g["tol"] * np.maximum(np.abs(got), np.abs(exp)))


@pytest.mark.parametrize("name", ["karate.csv", "dolphins.csv"])
def test_pylib_golden(golden, name):
    p = golden["pagerank_pylib"]
    s, d, w = og.read_csv(dataset_path(name))
    h, G = make_graph(s, d, w, transposed=True, renumber=False)
    v, pr = plc().pagerank(h, G, None, None, None, None, p["alpha"], p["epsilon"], p["max_iterations"], False)
    got = by_ext(v, pr)
    assert got == pytest.approx(np.asarray(p[name]), rel=1e-4)


def test_not_converged_raises():
    h, G = make_graph([0, 1, 2], [1, 2, 0], None, transposed=True, renumber=False)
    with pytest.raises(RuntimeError, match="failed to converge"):
        plc().pagerank(h, G, None, None, None, None, 0.85, 0.0, 3, False)


def test_invalid_alpha():
    h, G = make_graph([0, 1], [1, 0], None, transposed=True)
    with pytest.raises(ValueError, match="alpha"):
        plc().pagerank(h, G, None, None, None, None, 1.5, 1e-6, 100, False)


@functools.lru_cache(maxsize=None)
def rmat_graph(scale, weighted, symmetric=True, seed=42):
    """Generated once per module (the RMAT-20 edge lists are shared by several
    tests); callers must not modify the arrays."""
    s, d = rmat.rmat(scale, 16 << scale, seed=seed)
    w = rmat.rmat_weights(s.size, seed=seed + 1).astype(np.float64) if weighted else None
    if symmetric:
        s, d, w = og.symmetrize_dedup(s, d, w)
    return s, d, w


@pytest.mark.parametrize("scale,weighted,symmetric,renumber,transposed",
                         [(10, False, True, True, True), (12, False, True, True, True),
                          (12, True, True, True, True), (12, False, False, True, True),
                          (12, True, False, False, False), (13, False, True, False, True)])
def test_rmat_vs_oracle(scale, weighted, symmetric, renumber, transposed):
    s, d, w = rmat_graph(scale, weighted, symmetric)
    h, G = make_graph(s, d, None if w is None else w.astype(np.float32), transposed=transposed,
                      renumber=renumber, symmetric=symmetric)
    v, pr = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
    # oracle on the same vertex set
    og_g = og.create_graph(s, d, None if w is None else w.astype(np.float32), store_transposed=True,
                           renumber=renumber)
    ref = opr.pagerank_from_graph(og_g, alpha=0.85, epsilon=1e-6, max_iterations=500)
    ref_ext = np.zeros(int(og_g.number_map.max()) + 1)
    ref_ext[og_g.number_map] = ref
    got = by_ext(v, pr)
    vv = host(v)
    assert vv.size == og_g.num_vertices
    rel = np.abs(got[vv] - ref_ext[vv]) / ref_ext[vv]
    assert rel.max() < REL, rel.max()
    assert abs(got[vv].sum() - 1.0) < 1e-5


def test_rmat_float64_and_int64():
    s, d, w = rmat_graph(11, True)
    h, G = make_graph(s, d, w, transposed=True, renumber=True, symmetric=True, vdtype=np.int64,
                      wdtype=np.float64)
    v, pr = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-10, 1000, False)
    assert pr.dtype.is_floating_point and str(pr.dtype) == "torch.float64"
    og_g = og.create_graph(s, d, w, store_transposed=True, renumber=True)
    ref = opr.pagerank_from_graph(og_g, alpha=0.85, epsilon=1e-10, max_iterations=1000)
    ref_ext = np.zeros(int(og_g.number_map.max()) + 1)
    ref_ext[og_g.number_map] = ref
    vv = host(v)
    got = by_ext(v, pr)
    assert np.max(np.abs(got[vv] - ref_ext[vv]) / ref_ext[vv]) < 1e-9


def _fp64_vs_oracle(got, ref, it_gpu, it_ref, what):
    """fp64 at size: with the same iteration count the two differ only by rounding
    (the push's 2^-62 fixed point against fp64 sums), so 1e-10 relative; a
    quantisation of 2^-52 (fp32's scale) puts low-degree x~ terms (~2^-26 at RMAT-20)
    at ~1e-8 and fails it."""
    rel = np.abs(got - ref) / ref
    print(f"{what}: iterations gpu {it_gpu} oracle {it_ref}, max rel {rel.max():.3e}")
    assert it_gpu == it_ref
    assert rel.max() < 1e-10, rel.max()


def test_rmat20_float64_unit_weights_vs_compiled_oracle():
    """fp64 PageRank at RMAT-20 (symmetric, all-ones fp64 weights: the packed
    unweighted push with R = double) against the compiled fp64 oracle on the
    library's own CSC (internal ids), epsilon 1e-10."""
    import torch
    from oracle import cpu_native
    p = plc()
    h = p.ResourceHandle()
    n = 16 << 20
    s, d = p.generators.generate_rmat_edgelist(h, 20, n, 0.57, 0.19, 0.19, 42, False, True)
    s, d, _ = p.generators.symmetrize_dedup(h, s, d, None, True)
    w = torch.ones(s.numel(), dtype=torch.float64, device=s.device)
    G = p.SGGraph(h, p.GraphProperties(is_symmetric=True, is_multigraph=False), s, d, w, store_transposed=True,
                  renumber=True)
    v, pr = p.pagerank(h, G, None, None, None, None, 0.85, 1e-10, 1000, False)
    assert str(pr.dtype) == "torch.float64"
    it_gpu = h.last_iterations()
    off, idx, _ = G.adjacency(h, transposed=True)
    ref, it_ref = cpu_native.pagerank_f64(host(off).astype(np.int64), host(idx), 0.85, 1e-10, 1000, threads=8)
    _fp64_vs_oracle(host(pr), ref, it_gpu, it_ref, f"RMAT-20 fp64 unit weights V={ref.size} E={idx.numel()}")


def test_rmat18_float64_weighted_vs_oracle():
    """fp64 PageRank with random fp64 weights at RMAT-18 (the 32-bit entry + weight
    push, to_fixed<double>) against the numpy fp64 oracle, epsilon 1e-10."""
    s, d, w = rmat_graph(18, True)
    h, G = make_graph(s, d, w, transposed=True, renumber=True, symmetric=True, wdtype=np.float64)
    v, pr = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-10, 1000, False)
    it_gpu = h.last_iterations()
    og_g = og.create_graph(s, d, w, store_transposed=True, renumber=True)
    ref, it_ref = opr.pagerank_from_graph(og_g, alpha=0.85, epsilon=1e-10, max_iterations=1000,
                                          return_iterations=True)
    ref_ext = np.zeros(int(og_g.number_map.max()) + 1)
    ref_ext[og_g.number_map] = ref
    vv = host(v)
    _fp64_vs_oracle(by_ext(v, pr)[vv], ref_ext[vv], it_gpu, it_ref, "RMAT-18 fp64 weighted")


def test_initial_guess_and_precomputed_outw():
    s, d, _ = rmat_graph(10, False)
    h, G = make_graph(s, d, None, transposed=True, renumber=True, symmetric=True)
    v0, pr0 = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-8, 500, False)
    it_cold = h.last_iterations()
    # warm start from the converged answer converges at once
    v1, pr1 = plc().pagerank(h, G, None, None, v0, pr0, 0.85, 1e-6, 500, False)
    assert h.last_iterations() <= 2 < it_cold
    outw = np.bincount(s, minlength=int(max(s.max(), d.max())) + 1).astype(np.float32)
    verts = np.unique(np.concatenate([s, d])).astype(np.int32)
    v2, pr2 = plc().pagerank(h, G, verts, outw[verts], None, None, 0.85, 1e-8, 500, False)
    a, b = by_ext(v0, pr0), by_ext(v2, pr2)
    assert np.allclose(a, b, rtol=1e-6, atol=0)


def test_understated_precomputed_outw():
    """Precomputed out-weight sums below the graph's own take the pull kernel with
    fp64 sums: at 0.9 x the degrees the iteration still contracts (alpha / 0.9 < 1)
    to a fixed point whose total mass is ~2.7 -- matched against the oracle at 1e-6;
    at 0.5 x it diverges, and the call must fail to converge (as the oracle does)
    instead of reporting convergence on a wrapped or saturated sum."""
    s, d, _ = rmat_graph(10, False)
    h, G = make_graph(s, d, None, transposed=True, renumber=False, symmetric=True)
    V = int(max(s.max(), d.max())) + 1
    deg = np.bincount(s, minlength=V).astype(np.float64)
    verts = np.arange(V, dtype=np.int32)
    outw = (0.9 * deg).astype(np.float32)
    v, pr = plc().pagerank(h, G, verts, outw, None, None, 0.85, 1e-8, 500, False)
    ref = opr.pagerank(V, s, d, alpha=0.85, epsilon=1e-8, out_weight_sums=outw.astype(np.float64))
    got = by_ext(v, pr)
    live = ref > 0
    assert ref.sum() > 2.0
    assert np.max(np.abs(got[live] - ref[live]) / ref[live]) < REL
    with pytest.raises(opr.PageRankNotConverged):
        opr.pagerank(V, s, d, alpha=0.85, epsilon=1e-6, max_iterations=200,
                     out_weight_sums=(0.5 * deg))
    with pytest.raises(RuntimeError, match="converge"):
        plc().pagerank(h, G, verts, (0.5 * deg).astype(np.float32), None, None, 0.85, 1e-6, 200, False)


def test_repeat_is_bitwise_deterministic():
    s, d, _ = rmat_graph(12, False)
    h, G = make_graph(s, d, None, transposed=True, renumber=True, symmetric=True)
    r1 = host(plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)[1])
    r2 = host(plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)[1])
    assert np.array_equal(r1, r2)


def test_empty_and_edgeless_graph():
    h, G = make_graph([0, 3], [0, 3], None, transposed=True, renumber=False)  # self loops only
    v, pr = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 100, False)
    got = by_ext(v, pr)
    ref = opr.pagerank(4, [0, 3], [0, 3], None, 0.85, 1e-6, 100)
    assert np.allclose(got, ref, rtol=1e-6)


@pytest.mark.parametrize("weighted,symmetric,renumber", [(False, True, True), (True, False, False),
                                                        (False, False, False)])
def test_rmat_multi_window_push(weighted, symmetric, renumber):
    """Scale 20: > 2^19 sources (several source segments per window) and ~128
    destination windows of the push path (pagerank.hip), against the oracle and
    against the generic pull kernel (precomputed out-weights take that path)."""
    s, d, w = rmat_graph(20, weighted, symmetric)
    w32 = None if w is None else w.astype(np.float32)
    h, G = make_graph(s, d, w32, transposed=True, renumber=renumber, symmetric=symmetric)
    v, pr = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
    og_g = og.create_graph(s, d, w32, store_transposed=True, renumber=renumber)
    assert og_g.num_vertices > (1 << 19)
    ref = opr.pagerank_from_graph(og_g, alpha=0.85, epsilon=1e-6, max_iterations=500)
    ref_ext = np.zeros(int(og_g.number_map.max()) + 1)
    ref_ext[og_g.number_map] = ref
    got = by_ext(v, pr)
    vv = host(v)
    rel = np.abs(got[vv] - ref_ext[vv]) / ref_ext[vv]
    assert rel.max() < REL, rel.max()
    # generic pull path on the same graph
    n = int(ref_ext.size)
    wsum = np.zeros(n)
    np.add.at(wsum, s, 1.0 if w32 is None else w32.astype(np.float64))
    verts = vv.astype(np.int32)
    v2, pr2 = plc().pagerank(h, G, verts, wsum[verts].astype(np.float32), None, None, 0.85, 1e-6, 500, False)
    got2 = by_ext(v2, pr2)
    assert np.max(np.abs(got2[vv] - got[vv]) / got[vv]) < REL


@pytest.mark.parametrize("nv,ne", [((1 << 22) + 37, 200_000), ((1 << 21) - 5, 300_000), (130, 900)])
def test_sparse_wide_push(nv, ne):
    """Window geometry edge cases of the push schedule (pagerank.hip
    build_push_from_coo): 4M ids with 200K edges (8K-destination windows, a
    partial last window) put ~400 entries spread over 4M sources in each window,
    so units are split at aligned 2^19 source blocks; 2M ids (4K windows, units
    split at 2^20 blocks); a graph of one window.  Not renumbered, so isolated ids
    are vertices too."""
    rng = np.random.default_rng(nv)
    s = rng.integers(0, nv, ne).astype(np.int32)
    d = rng.integers(0, nv, ne).astype(np.int32)
    s[0], d[0] = nv - 1, 0  # the full id range is present
    pairs = np.unique(s.astype(np.int64) * nv + d)
    s, d = (pairs // nv).astype(np.int32), (pairs % nv).astype(np.int32)
    h, G = make_graph(s, d, None, transposed=True, renumber=False, symmetric=False)
    v, pr = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
    got = by_ext(v, pr)
    ref = opr.pagerank(nv, s, d, None, 0.85, 1e-6, 500)
    rel = np.abs(got[:nv] - ref) / ref
    assert rel.max() < REL, rel.max()


@pytest.mark.parametrize("scale,renumber", [(12, True), (20, True), (20, False)])
def test_packed_entries_bitwise_equal_plain(scale, renumber):
    """The 16-bit packed push entries (pagerank.hip push_body16: source deltas, jump
    entries, per-wave-segment bases) must give the same fixed-point sums -- so the
    same bits -- as the 32-bit entries (option pr_packed = 0)."""
    s, d, _ = rmat_graph(scale, False, True)
    h, G = make_graph(s, d, None, transposed=True, renumber=renumber, symmetric=True)
    r_packed = host(plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)[1])
    it = h.last_iterations()
    h2, G2 = make_graph(s, d, None, transposed=True, renumber=renumber, symmetric=True, options={"pr_packed": 0})
    r_plain = host(plc().pagerank(h2, G2, None, None, None, None, 0.85, 1e-6, 500, False)[1])
    assert h2.last_iterations() == it
    assert np.array_equal(r_packed, r_plain)


def _star_plus_ring(n_leaves):
    """Vertex 0 points to n_leaves leaves and has no in-edges, so its x~ =
    pr / outdeg ~ 0.15 / V / V falls below 2^-39: enc_fixed's rounding branch.
    A ring over the leaves keeps them non-dangling."""
    leaves = np.arange(1, n_leaves + 1, dtype=np.int32)
    s = np.concatenate([np.zeros(n_leaves, np.int32), leaves])
    d = np.concatenate([leaves, np.roll(leaves, -1)])
    return s, d


@pytest.mark.parametrize("graph", ["rmat20", "star"])
def test_encoded_x_bitwise_equal_float(graph):
    """The single-GPU fp32 packed push reads x~ as enc_fixed words (pagerank.hip:
    M << s, tiny values rounded to nearest-even once per vertex in the apply); it
    must give the same bits as the float x~ converted per entry (pr_enc = 0),
    and stay within REL of the oracle."""
    if graph == "rmat20":
        s, d, _ = rmat_graph(20, False, True)
        sym, nv = True, None
    else:
        s, d = _star_plus_ring(1 << 20)
        sym, nv = False, (1 << 20) + 1
    h, G = make_graph(s, d, None, transposed=True, renumber=True, symmetric=sym)
    v, pr = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
    r_enc = host(pr)
    it = h.last_iterations()
    h2, G2 = make_graph(s, d, None, transposed=True, renumber=True, symmetric=sym, options={"pr_enc": 0})
    r_flt = host(plc().pagerank(h2, G2, None, None, None, None, 0.85, 1e-6, 500, False)[1])
    assert h2.last_iterations() == it
    assert np.array_equal(r_enc, r_flt)
    if nv is not None:
        got = by_ext(v, pr)
        ref = opr.pagerank(nv, s, d, None, 0.85, 1e-6, 500)
        assert (np.abs(got[:nv] - ref) / ref).max() < REL



@pytest.mark.parametrize("scale", [12, 20])
def test_unit_weights_take_unweighted_push(scale):
    """All-ones fp32 weights (cugraph.Graph's unweighted graphs, simpleGraph.py:840-843)
    are detected and run the unweighted 16-bit push: the ranks are bitwise those of
    the same graph without weights; the entry-weight push (pr_unit_w = 0) agrees
    within 1e-6 relative of the oracle."""
    s, d, _ = rmat_graph(scale, False, True)
    ones = np.ones(s.size, np.float32)
    h, G = make_graph(s, d, None, transposed=True, symmetric=True)
    v0, r0 = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
    hw, Gw = make_graph(s, d, ones, transposed=True, symmetric=True)
    v1, r1 = plc().pagerank(hw, Gw, None, None, None, None, 0.85, 1e-6, 500, False)
    assert np.array_equal(host(v0), host(v1)) and np.array_equal(host(r0), host(r1))
    assert hw.last_iterations() == h.last_iterations()
    hq, Gq = make_graph(s, d, ones, transposed=True, symmetric=True, options={"pr_unit_w": 0})
    v2, r2 = plc().pagerank(hq, Gq, None, None, None, None, 0.85, 1e-6, 500, False)
    assert np.array_equal(host(v0), host(v2))
    rel = np.abs(host(r2).astype(np.float64) - host(r0)) / host(r0)
    assert rel.max() < 2e-6
    # a weight that is not 1 keeps the entry-weight push
    if scale != 12:
        return
    w = ones.copy()
    w[0] = 2.0  # one direction only: the graph is no longer symmetric
    h3, G3 = make_graph(s, d, w, transposed=True, symmetric=False)
    v3, r3 = plc().pagerank(h3, G3, None, None, None, None, 0.85, 1e-6, 500, False)
    og_g = og.create_graph(s, d, w, store_transposed=True, renumber=True)
    ref = opr.pagerank_from_graph(og_g, alpha=0.85, epsilon=1e-6, max_iterations=500)
    ref_ext = np.zeros(int(og_g.number_map.max()) + 1)
    ref_ext[og_g.number_map] = ref
    got = by_ext(v3, r3)
    vv = host(v3)
    assert (np.abs(got[vv] - ref_ext[vv]) / ref_ext[vv]).max() < REL


@pytest.mark.parametrize("scale", [12, 20])
def test_window_bits_bitwise_equal(scale):
    """4K, 8K, 16K and 32K-destination windows (pr_win_bits 12 / 13 / 14 / 15; 14 and
    15 run one 128 KB-LDS block per CU, 15 in 32-bit words with carries) sum the same
    fixed-point terms: the same bits.  (15 with 32-bit entries is built as 14.)"""
    s, d, _ = rmat_graph(scale, False, True)
    out = []
    for wb in (12, 13, 14, 15):
        for packed in (1, 0):
            h, G = make_graph(s, d, None, transposed=True, symmetric=True,
                              options={"pr_win_bits": wb, "pr_packed": packed})
            v, r = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
            out.append((host(v), host(r), h.last_iterations()))
    for o in out[1:]:
        assert o[2] == out[0][2]
        assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1])


def _empty_window_graph():
    """Not renumbered, 16K windows: ids >= 2^15 only send (no in-edges), so windows 2
    and 3 have no push items and are applied by the last window's block."""
    rng = np.random.default_rng(3)
    n_lo, n = 1 << 15, (1 << 15) + (1 << 14) + 100
    hi = np.arange(n_lo, n, dtype=np.int32)
    s = np.concatenate([hi, np.arange(n_lo, dtype=np.int32), rng.integers(0, n_lo, 200_000).astype(np.int32)])
    d = np.concatenate([rng.integers(0, n_lo, hi.size).astype(np.int32), np.roll(np.arange(n_lo, dtype=np.int32), 1),
                        rng.integers(0, n_lo, 200_000).astype(np.int32)])
    pairs = np.unique(s.astype(np.int64) * n + d)
    pairs = pairs[pairs // n != pairs % n]
    return (pairs // n).astype(np.int32), (pairs % n).astype(np.int32), n


@pytest.mark.parametrize("graph,wb", [("rmat20", 14), ("rmat20", 15), ("empty_windows", 14)])
def test_fused_apply_bitwise_equal(graph, wb):
    """The push with the apply fused in (pagerank.hip fused_finish: the block that
    finishes a window applies it, from LDS for whole-window items; the last one
    applies the windows without items and updates the state) gives the same bits
    and iteration count as the separate k_pr_apply (pr_fuse = 0), with and
    without whole-window items (pr_whole = 0)."""
    if graph == "rmat20":
        s, d, _ = rmat_graph(20, False, True)
        kw = dict(renumber=True, symmetric=True)
        n = None
    else:
        s, d, n = _empty_window_graph()
        kw = dict(renumber=False, symmetric=False)
    out = []
    for fuse, whole in ((1, 1), (0, 1), (1, 0)):
        h, G = make_graph(s, d, None, transposed=True, **kw,
                          options={"pr_win_bits": wb, "pr_fuse": fuse, "pr_whole": whole})
        v, r = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        # a second call on the same schedule: queue heads and window counts were reset
        _, r2 = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        assert np.array_equal(host(r), host(r2))
        out.append((host(v), host(r), h.last_iterations()))
    for o in out[1:]:
        assert o[2] == out[0][2]
        assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1])
    if n is not None:
        got = np.zeros(n)
        got[out[0][0]] = out[0][1]
        ref = opr.pagerank(n, s, d, None, 0.85, 1e-6, 500)
        assert (np.abs(got[:n] - ref) / ref).max() < REL


@pytest.mark.parametrize("scale,wb", [(12, 14), (20, 14), (20, 0), (18, 12), (20, 15)])
def test_fast_symmetric_build_bitwise_equal(scale, wb):
    """The one-word-key schedule build of symmetric unweighted graphs (pagerank.hip
    build_push_packed_sym: keys from the out-edge adjacency, a keys-only sort of the
    window bits, units from the window starts) gives the same ranks and iteration
    counts as the general build (option pr_fast_build = 0), with and without source
    bands."""
    s, d, _ = rmat_graph(scale, False, True)
    out = []
    for fast, cut in ((1, 0), (0, 0), (1, 4096), (0, 4096)):
        h, G = make_graph(s, d, None, transposed=True, renumber=True, symmetric=True,
                          options={"pr_win_bits": wb, "pr_fast_build": fast, "pr_band_cut": cut})
        v, r = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        out.append((host(v), host(r), h.last_iterations()))
    for o in out[1:]:
        assert o[2] == out[0][2]
        assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1])


@pytest.mark.parametrize("graph", ["rmat20", "empty_windows", "star"])
def test_banded_push_bitwise_equal(graph):
    """Source bands (pagerank.hip banded_finish: every 16K window's entries split at a
    source cut into two virtual windows, the stream and the queues band-major, a
    window applied by the last of its items from its LDS and the other band's plane)
    give the same bits and iteration count as the unbanded push, for cuts that put
    most entries in either band, on the first (calibrating) and a later call."""
    if graph == "rmat20":
        s, d, _ = rmat_graph(20, False, True)
        kw = dict(renumber=True, symmetric=True)
    elif graph == "star":
        s, d = _star_plus_ring(300_000)
        kw = dict(renumber=True, symmetric=False)
    else:
        s, d, _ = _empty_window_graph()
        kw = dict(renumber=False, symmetric=False)
    out = []
    for cut in (0, 64, 4096, 65536, 262144):
        h, G = make_graph(s, d, None, transposed=True, **kw, options={"pr_win_bits": 14, "pr_band_cut": cut})
        v, r = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        v2, r2 = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        assert np.array_equal(host(r), host(r2)) and h.last_iterations() > 0
        out.append((host(v), host(r), h.last_iterations()))
    for o in out[1:]:
        assert o[2] == out[0][2]
        assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1])


@pytest.mark.parametrize("graph", ["rmat12", "rmat20", "star"])
def test_hub_lds_bitwise_equal(graph):
    """The 16K-window push that reads the hubs' x~ from LDS (pagerank.hip push_body16
    HUB: segments whose sources are all below the staged count) gives the same bits
    as gathering every x~ from global memory (pr_hub = 0), with encoded and plain
    float x~.  RMAT-12 has fewer vertices than the LDS holds (every segment reads
    LDS); the star graph has long runs of one hub source."""
    if graph == "star":
        s, d = _star_plus_ring(300_000)
    else:
        s, d, _ = rmat_graph(int(graph[4:]), False, True)
    out = []
    for hub, enc in ((1, 1), (0, 1), (1, 0)):
        h, G = make_graph(s, d, None, transposed=True, symmetric=graph != "star",
                          options={"pr_win_bits": 14, "pr_hub": hub, "pr_enc": enc})
        v, r = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        out.append((host(v), host(r), h.last_iterations()))
    for o in out[1:]:
        assert o[2] == out[0][2]
        assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1])


@pytest.mark.parametrize("deal", ["xcd", "global"])
def test_calibrated_queues_bitwise_equal(deal):
    """Measured-cost queues (pagerank.hip calibrate_queues): the first call on a
    schedule records every item's duration and re-deals the queues after its first
    chunk; that call, a later one on the re-dealt queues, and entry-dealt queues
    (pr_calib = 0) give the same bits and iteration counts, for 4K (one queue of
    tiles, re-sorted longest-first), 8K and 16K windows."""
    s, d, _ = rmat_graph(20, False, True)
    for wb in (12, 13, 14):
        out = []
        for calib in (1, 0):
            h, G = make_graph(s, d, None, transposed=True, symmetric=True,
                              options={"pr_win_bits": wb, "pr_calib": calib, "pr_deal_global": int(deal == "global")})
            for _ in range(2):  # calibrating call, then a call on the re-dealt queues
                v, r = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
                out.append((host(v), host(r), h.last_iterations()))
        for o in out[1:]:
            assert o[2] == out[0][2]
            assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1])


def _outw_host(G, h):
    """(number map, CSR offsets, CSR weights) in internal order, and the library's sums."""
    v, _ = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-2, 500, False)
    got = host(G.out_weight_sums(h))
    off, _, w = G.adjacency(h, transposed=False)
    return host(v), host(off).astype(np.int64), host(w).astype(np.float64), got


@pytest.mark.parametrize("case", ["star_exact", "aligned_rows", "rmat20_uniform", "fp64_weights"])
def test_out_weight_sums_tiled(case):
    """compute_out_weight_sums (pagerank_impl.cuh:158-164) over edge tiles
    (graph_build.hip k_row_sums_tiles / k_row_sums_spill): rows spanning many 2048-edge
    tiles (a 300K-edge hub), rows ending exactly on tile boundaries, zero-degree rows
    between and after the edges.  Weights that are multiples of 1/8 make every fp64
    sum exact, so those must be bitwise the numpy sums; uniform weights within one
    fp32 ulp."""
    rng = np.random.default_rng(5)
    wdtype = np.float32
    if case == "star_exact":
        n = 300_000
        leaves = np.arange(1, n + 1)
        s = np.concatenate([np.zeros(n, np.int64), leaves, leaves])
        d = np.concatenate([leaves, np.roll(leaves, -1), np.zeros(n, np.int64)])
        w = rng.integers(1, 64, s.size) / 8.0
        renumber, sym = True, False
    elif case == "aligned_rows":
        # out-degrees 2048, 4096, 1, 0 (isolated ids 3..9 never appear as sources), 2047, 2049 ...
        degs = [2048, 4096, 1, 0, 0, 0, 0, 0, 0, 0, 2047, 2049, 6144, 1, 2048]
        s = np.concatenate([np.full(k, i, np.int64) for i, k in enumerate(degs)])
        nv = 20000
        d = np.concatenate([rng.choice(np.arange(20, nv), k, replace=False) for k in degs])
        d[0] = nv - 1  # the id range reaches nv - 1: trailing ids without out-edges
        w = rng.integers(1, 64, s.size) / 8.0
        renumber, sym = False, False
    else:
        s, d, _ = rmat_graph(20, False, True)
        w = rng.random(s.size)
        renumber, sym = True, True
        if case == "fp64_weights":
            wdtype = np.float64
            w = rng.integers(1, 1 << 20, s.size) / 1024.0
    h, G = make_graph(s, d, w, transposed=False, renumber=renumber, symmetric=sym, wdtype=wdtype)
    v, off, ww, got = _outw_host(G, h)
    want = np.add.reduceat(np.concatenate([ww, [0.0]]), off[:-1]) * (off[1:] > off[:-1])
    want = want.astype(wdtype)
    assert got.dtype == wdtype and got.shape == want.shape
    if case == "rmat20_uniform":
        rel = np.abs(got.astype(np.float64) - want) / np.maximum(want, 1e-30)
        assert rel.max() <= 1.2e-7 and (got == want).mean() > 0.9999
    else:
        assert np.array_equal(got, want)


@pytest.mark.parametrize("n", [4000, 200_000])
def test_wide_window_carries_bitwise_equal(n):
    """32K windows sum in 32-bit LDS words (push_body16, WB = 15): a small graph has
    large x~ terms (1 / V, above 2^-20: high words counted in the carry array) and
    destinations whose sums wrap the 32-bit word many times per window (every carry
    counted).  Same bits and iterations as the 64-bit-word 16K windows, fused and
    separate apply, and a second call on the cached schedule (carries cleared)."""
    rng = np.random.default_rng(11)
    m = 40 * n
    s = rng.integers(0, n, m).astype(np.int32)
    d = (rng.integers(0, n, m) // rng.integers(1, 50, m)).astype(np.int32)  # skewed to low ids
    pairs = np.unique(np.concatenate([s.astype(np.int64) * n + d, d.astype(np.int64) * n + s]))
    pairs = pairs[pairs // n != pairs % n]
    s, d = (pairs // n).astype(np.int32), (pairs % n).astype(np.int32)
    out = []
    for wb, fuse in ((14, 1), (15, 1), (15, 0)):
        h, G = make_graph(s, d, None, transposed=True, renumber=True, symmetric=True,
                          options={"pr_win_bits": wb, "pr_fuse": fuse})
        v, r = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        _, r2 = plc().pagerank(h, G, None, None, None, None, 0.85, 1e-6, 500, False)
        assert np.array_equal(host(r), host(r2))
        out.append((host(v), host(r), h.last_iterations()))
    for o in out[1:]:
        assert o[2] == out[0][2]
        assert np.array_equal(o[0], out[0][0]) and np.array_equal(o[1], out[0][1])
    og_g = og.create_graph(s, d, None, store_transposed=True, renumber=True)
    ref = np.zeros(n)
    ref[og_g.number_map] = opr.pagerank_from_graph(og_g, alpha=0.85, epsilon=1e-6, max_iterations=500)
    vv = out[0][0]
    got = np.zeros(n)
    got[vv] = out[0][1]
    assert (np.abs(got[vv] - ref[vv]) / ref[vv]).max() < REL

#!/usr/bin/env python3
"""Benchmark: PageRank edges/s + BFS MTEPS on Graph500 R-MAT scale 24, MI355X.

BASELINE.json metric: "PageRank edges/sec + BFS MTEPS on RMAT-24 at 1/2/4/8 MI355X".
Headline (``value``): PageRank on RMAT scale-24 -- symmetrised + deduplicated,
unweighted, fp32, alpha 0.85, epsilon 1e-6 -- on the resident graph.  A "step" is
one complete ``cugraph_pagerank`` call (power iteration to convergence).
value = stored edges x PageRank iterations x steps / timed seconds (whole job; the
same graph at every N, so ``scaling`` is "strong").

Extra fields on the same JSON line:
  roofline         -- the PageRank iteration: algorithmic bytes/iteration 4E + 16V
                       / average iteration time from HIP events
                      recorded on the library's stream around each chunk of
                      iterations in the timed region; peak 8 TB/s; traffic = HBM
                      bytes per iteration from rocprofv3 PMC passes; copy_ceiling =
                      a measured 16-B-per-lane copy kernel (ext.h).
  cpu_baseline     -- (N=1) NetworkX's PageRank loop restated on scipy (the port of
                      nx.pagerank's _pagerank_scipy, fp64, 1 core) on the SAME
                      RMAT-24 graph for a few iterations; plus the compiled C
                      restatement of the reference CPU reference (1 thread and
                      OpenMP), nx.pagerank itself on the largest sample that stays
                      bounded, and the host's core count.
  pagerank_rmat22  -- (N=1) configs[1]: the same measurement on RMAT-22.
  pagerank_rmat26  -- (N=8) configs[3]: RMAT-26 on the 2D partition.
  pagerank_alt_grid-- (N>1) the headline graph on the other R x C grid (1 x P).
  pagerank_overlap_k4 -- (N>1, several grid rows) the headline graph with the
                      column reduce-scatter overlapped in 4 row chunks, and whether
                      its ranks equal the default's bit for bit.
  bfs              -- configs[2]: RMAT-24 BFS, Graph500 MTEPS (harmonic mean over
                      8 roots), its roofline (4E_cc + 16V_cc per traversal) and PMC
                      traffic, and CPU baselines (NetworkX on a bounded sample,
                      compiled C restatement on the same graph).
  sssp             -- (N=1) SSSP (near-far) on the BFS graph with uniform [0, 1)
                      weights from 4 roots: MTEPS, rounds, PMC traffic, and the
                      compiled near-far restatement as CPU baseline.
  louvain          -- configs[4]: Louvain time-to-solution on RMAT 23 + log2(N)
                      (RMAT-26 at 8 GPUs), uniform weights.

Multi-GPU (--gpus N, launched by torch.distributed.run, one process per GPU): every
rank generates the same edge list, keeps its 1/N slice, and the MG graph is built
collectively (cugraph_mg_graph_create: hash owners, degree renumbering, 2D R x C
edge blocks, R x C = the reference's grid by default); PageRank and BFS run over
RCCL communicators created inside libcugraph_c (pylibcugraph.comms.init_rccl).
torch.distributed (gloo) carries only the RCCL unique id, the timing barrier and
the max over ranks.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import math
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# (k_bfs_head, the bottom-up probe's per-graph head table, is matched first and kept out
# of the per-traversal sums: built once per graph, like the PageRank push schedule)
BFS_KERNELS = ("k_bfs_head", "k_topdown", "k_bu_probe", "k_bu_residual", "k_bottomup", "k_mark_queues",
               "k_bitmap_to_queues", "k_bfs_init_sources", "k_finish_pred", "k_sources_to_bitmap", "k_bfs_")
BFS_PER_GRAPH = ("k_bfs_head",)
PR_KERNELS = ("k_pr_push", "k_pr_apply")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def release_caches(p):
    """Between legs: torch's cached blocks and libcugraph_c's caching allocator."""
    import torch
    torch.cuda.synchronize()
    p.trim_device_cache()
    torch.cuda.empty_cache()


def barrier(args):
    if args.world > 1:
        import torch.distributed as dist
        dist.barrier()


def _allreduce(args, v, op):
    if args.world == 1:
        return v
    import torch
    import torch.distributed as dist
    x = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(x, op=op)
    return float(x[0])


def max_over_ranks(args, t):
    import torch.distributed as dist
    return _allreduce(args, t, dist.ReduceOp.MAX) if args.world > 1 else t


def sum_over_ranks(args, v):
    import torch.distributed as dist
    return _allreduce(args, v, dist.ReduceOp.SUM) if args.world > 1 else v


def host_info(threads):
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "model": model, "threads_used": threads}


def omp_threads():
    """Threads for the OpenMP baseline: the process's CPU share (16 on a one-GPU box:
    OMP_NUM_THREADS is set there), never more than the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(aff, env if env > 0 else 16))


# ----------------------------------------------------------------------------- graphs
def build_rmat_graph(p, h, scale, seed=42, weighted=False, transposed=True, want_roots=0, mg=None):
    """Device R-MAT -> symmetrise + dedup (cugraph.Graph preprocessing) -> graph.
    weighted: False (no weights at the C ABI), True (uniform [0, 1) fp32, seed + 1) or
    "ones" (all-ones fp32, the reference Python path's unweighted graph).
    mg = (rank, world): every rank makes the same edge list and passes its slice to
    the collective MGGraph build."""
    import numpy as np
    import torch
    n = 16 << scale
    s, d = p.generators.generate_rmat_edgelist(h, scale, n, 0.57, 0.19, 0.19, seed, False, True)
    if weighted == "ones":  # what cugraph.Graph attaches to an unweighted edge list (simpleGraph.py:840-843)
        w = torch.ones(n, dtype=torch.float32, device=s.device)
    else:
        w = p.generators.generate_edge_weights(h, n, seed + 1) if weighted else None
    s, d, w = p.generators.symmetrize_dedup(h, s, d, w, True)
    props = p.GraphProperties(is_symmetric=True, is_multigraph=False)
    roots, deg = None, None
    if want_roots:
        # Graph500 root sampling: vertices with degree > 0 (every edge source has one)
        rng = np.random.default_rng(seed)
        pick = torch.as_tensor(rng.integers(0, s.numel(), size=4 * want_roots), device=s.device)
        roots = list(dict.fromkeys(s[pick].cpu().numpy().tolist()))[:want_roots]
    if mg is None:
        g = p.SGGraph(h, props, s, d, w, store_transposed=transposed, renumber=True)
    else:
        rank, world = mg
        E = s.numel()
        if want_roots:
            deg = torch.bincount(s.to(torch.int64), minlength=1 << scale)  # degree by external id
        lo, hi = rank * E // world, (rank + 1) * E // world
        g = p.MGGraph(h, props, s[lo:hi].contiguous(), d[lo:hi].contiguous(),
                      None if w is None else w[lo:hi].contiguous(), store_transposed=transposed, num_edges=E)
    del s, d, w
    torch.cuda.synchronize()
    return g, roots, deg


# ----------------------------------------------------------------------------- PageRank
def pagerank_leg(p, args, scale, steps, warmup, ctx=None, weighted=False, options=None):
    import torch
    h = p.ResourceHandle(ctx.ptr if ctx else None)
    for k, v in (options or {}).items():  # measurement / A-B switches (include/cugraph_amd/ext.h)
        h.set_option(k, v)
    # module load (the code objects of every kernel on the path) off the clock: PageRank
    # on a tiny graph of the same kind, once per window size the big graphs use (16K and
    # 32K windows are picked by size: forced here on the tiny graph, then the leg's own
    # options restored), so first_call_ms is the graph's own cost
    for wb in (0, 14, 15):
        if wb:
            h.set_option("pr_win_bits", wb)
        small, _, _ = build_rmat_graph(p, h, 10, weighted=weighted, mg=args.mg)
        p.pagerank(h, small, None, None, None, None, args.alpha, args.epsilon, 500, False)
        del small
    h.set_option(None, 0)
    for k, v in (options or {}).items():
        h.set_option(k, v)
    barrier(args)
    t0 = time.perf_counter()
    g, _, _ = build_rmat_graph(p, h, scale, weighted=weighted, mg=args.mg)
    build_s = max_over_ranks(args, time.perf_counter() - t0)
    V, E = g.number_of_vertices(), g.number_of_edges()
    log(f"[bench] pagerank RMAT-{scale}: V={V} E={E} (build {build_s:.2f}s)")
    # first call on the fresh graph: out-weight sums, push schedule (window sort, packing,
    # work items) and the calibration chunk are once-per-graph work inside it
    torch.cuda.synchronize()
    barrier(args)
    t0 = time.perf_counter()
    p.pagerank(h, g, None, None, None, None, args.alpha, args.epsilon, 500, False)
    torch.cuda.synchronize()
    first_ms = max_over_ranks(args, time.perf_counter() - t0) * 1e3
    first_iters = h.last_iterations()
    for _ in range(max(warmup - 1, 0)):
        p.pagerank(h, g, None, None, None, None, args.alpha, args.epsilon, 500, False)
    torch.cuda.synchronize()
    iters, kms, klaunch = [], 0.0, 0
    h.set_profiling(True)
    barrier(args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        p.pagerank(h, g, None, None, None, None, args.alpha, args.epsilon, 500, False)
        iters.append(h.last_iterations())
        kms += h.last_hot_kernel_ms()
        klaunch += h.last_hot_kernel_launches()
    torch.cuda.synchronize()
    barrier(args)
    t = max_over_ranks(args, time.perf_counter() - t0)
    h.set_profiling(False)
    # the first call on the next fresh graph of this size (a new graph object of the same
    # edges): what every further graph costs once the process has run one -- the first
    # graph's first call also pays the one-time loads of the kernels only this size uses
    # and the allocator's first hipMallocs of its block sizes
    g2, _, _ = build_rmat_graph(p, h, scale, weighted=weighted, mg=args.mg)
    torch.cuda.synchronize()
    barrier(args)
    t1 = time.perf_counter()
    p.pagerank(h, g2, None, None, None, None, args.alpha, args.epsilon, 500, False)
    torch.cuda.synchronize()
    next_ms = max_over_ranks(args, time.perf_counter() - t1) * 1e3
    del g2
    value = E * sum(iters) / t
    # algorithmic bytes of one rank's share: (4E + 16V) / N, +4E when the
    # push reads edge weights -- not for all-ones weights, which run the unweighted push
    # unless the option pr_unit_w = 0 forces the entry-weight push
    reads_w = bool(weighted) and (weighted != "ones" or (options or {}).get("pr_unit_w", 1) == 0)
    bytes_per_iter = ((8 if reads_w else 4) * E + 16 * V) / args.world
    avg_ms = kms / max(klaunch, 1)
    achieved = bytes_per_iter / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    log(f"[bench] pagerank RMAT-{scale}: {value:.4g} edges/s, iters {iters}, {avg_ms:.4f} ms/iter, "
        f"{achieved:.1f} GB/s algorithmic")
    return dict(h=h, g=g, V=V, E=E, t=t, iters=iters, value=value, avg_ms=avg_ms, achieved=achieved,
                bytes_per_iter=bytes_per_iter, build_s=build_s, scale=scale, steps=steps, first_ms=first_ms,
                next_graph_first_ms=next_ms,
                first_iters=first_iters, steady_ms=t / steps * 1e3, reads_w=reads_w)


def pagerank_summary(r, args, grid=None):
    """The JSON object of one PageRank leg (secondary legs)."""
    return {"scale": r["scale"], "vertices": r["V"], "edges": r["E"], "value": r["value"], "unit": "edges/s",
            "ms_per_step": r["t"] / r["steps"] * 1e3, "iterations": r["iters"],
            "graph_build_s": round(r["build_s"], 3), "grid": grid, "first_call_ms": round(r["first_ms"], 3),
            "next_graph_first_call_ms": round(r["next_graph_first_ms"], 3),
            "push_reads_weights": r["reads_w"],
            "roofline": {"bound": "hbm", "achieved": r["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": r["achieved"] / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": r["bytes_per_iter"],
                         "avg_kernel_ms": r["avg_ms"]}}


def overlap_leg(p, args, mg_ref, C):
    """N > 1 with several grid rows: the headline graph with the column reduce-scatter
    overlapped with the push in K = 4 row chunks (option mg_chunks; the default is one
    chunk), timed like the headline and checked bitwise equal to the
    default's ranks on every rank (same graph, same partition: the sums are integer)."""
    import torch
    r2 = pagerank_leg(p, args, args.scale, args.steps, args.warmup, args.ctx, options={"mg_chunks": 4})
    v2, x2 = p.pagerank(r2["h"], r2["g"], None, None, None, None, args.alpha, args.epsilon, 500, False)
    same = (torch.equal(v2, mg_ref[0]) and torch.equal(x2.view(torch.int32), mg_ref[1])
            and r2["h"].last_iterations() == mg_ref[2])
    bad = int(sum_over_ranks(args, 0.0 if same else 1.0))
    out = pagerank_summary(r2, args, grid_name(args, C) + ", mg_chunks 4")
    out["bitwise_equal_to_default"] = bad == 0
    out["ranks_differing"] = bad
    del v2, x2, r2
    return out


# ----------------------------------------------------------------------------- PMC traffic
def pmc_pass(ctr, child_args, kernels):
    """One rocprofv3 --pmc pass over a child bench process; returns
    {kernel-prefix: [values per launch]} in KiB (MI355X_MICROARCH.md: FETCH_SIZE /
    WRITE_SIZE, one counter per pass since they cannot share one)."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        raise RuntimeError("rocprofv3 not found")
    env = dict(os.environ, TMPDIR="/tmp")
    with tempfile.TemporaryDirectory(dir="/tmp") as d:
        cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__)] + child_args
        r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           timeout=300)
        if r.returncode != 0:
            raise RuntimeError(f"rocprofv3 {ctr} rc={r.returncode}: {r.stderr.decode()[-300:]}")
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows += list(csv.DictReader(open(f)))
    out = {k: [] for k in kernels}
    for x in rows:
        for k in kernels:
            if k in x["Kernel_Name"]:
                out[k].append(float(x["Counter_Value"]))
                break
    return out


def pagerank_traffic(args):
    """HBM bytes per PageRank iteration (k_pr_push + k_pr_apply): 2 x FETCH_SIZE
    (gfx950 tallies 128-B requests at 64 B) + WRITE_SIZE, KiB -> bytes.  Launches
    after convergence (no-ops) are skipped."""
    per = {}
    child = ["--traffic-child", "pagerank", "--scale", str(args.scale)]
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = pmc_pass(ctr, child, PR_KERNELS)
        tot = 0.0
        for k, v in vals.items():
            if not v:
                if k == "k_pr_apply":
                    continue
                raise RuntimeError(f"no {k} launches under rocprofv3")
            live = [x for x in v if x > 0.01 * max(v)]
            tot += sum(live) / len(live)
        per[ctr] = tot
    return (2.0 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024.0, per


def bfs_traffic(args, traversals):
    """HBM bytes per BFS traversal (the BFS kernels of the child's traversals, without
    the per-graph head table), the per-kernel split (KiB per traversal) of each counter,
    and the head table's bytes (per graph)."""
    per, by_kernel, graph = {}, {}, {}
    child = ["--traffic-child", "bfs", "--bfs-scale", str(args.bfs_scale), "--bfs-roots", str(args.bfs_roots)]
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = pmc_pass(ctr, child, BFS_KERNELS)
        per[ctr] = sum(sum(v) for k, v in vals.items() if k not in BFS_PER_GRAPH) / traversals
        by_kernel[ctr] = {k: round(sum(v) / traversals, 1) for k, v in vals.items() if v and k not in BFS_PER_GRAPH}
        graph[ctr] = {k: round(sum(v), 1) for k, v in vals.items() if v and k in BFS_PER_GRAPH}
    per["per_kernel_kib"] = by_kernel
    per["per_graph_kib"] = graph
    return (2.0 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024.0, per


# ----------------------------------------------------------------------------- CPU baselines
def pagerank_cpu_baseline(p, r, args):
    """SURVEY.md §8d.  Primary: NetworkX's PageRank loop (_pagerank_scipy restated on
    scipy, fp64, 1 core) on the same graph, a few iterations.  Secondary: the compiled
    C restatement of the reference's CPU reference (1 thread, OpenMP) and nx.pagerank
    itself on a bounded sample."""
    import numpy as np
    from oracle.baseline import networkx_pagerank, pagerank_scipy_iterations
    off, idx, _ = r["g"].adjacency(r["h"], transposed=True)
    off, idx = off.cpu().numpy().astype(np.int64), idx.cpu().numpy()
    V, E = r["V"], r["E"]
    t, eps = pagerank_scipy_iterations(off, idx, V, iterations=args.cpu_iters)
    T = omp_threads()
    out = {"value": eps, "unit": "edges/s", "cores": 1, "kind": "port",
           "sample": f"{args.cpu_iters} NetworkX-style scipy power iterations (nx.pagerank's _pagerank_scipy loop, "
                     f"fp64, 1 thread) on the same RMAT-{r['scale']} graph ({t:.1f}s); graph build excluded as on "
                     "the GPU",
           "host": host_info(T)}
    try:
        from oracle import cpu_native
        t1, _ = cpu_native.pagerank(off, idx, args.cpu_iters, args.alpha, threads=1)
        tn, _ = cpu_native.pagerank(off, idx, args.cpu_iters, args.alpha, threads=T)
        out["compiled"] = {
            "kind": "port", "source": "oracle/cpu_baseline.c (pagerank_test.cpp:43-130 restated, fp32)",
            "single_thread": {"value": E * args.cpu_iters / t1, "unit": "edges/s", "cores": 1},
            "openmp": {"value": E * args.cpu_iters / tn, "unit": "edges/s", "cores": T},
            "sample": f"{args.cpu_iters} iterations on the same RMAT-{r['scale']} graph"}
    except Exception as e:  # noqa: BLE001
        out["compiled"] = {"error": repr(e)[:200]}
    del off, idx
    try:
        sc = args.nx_pagerank_scale
        tb, tp, ne, it = networkx_pagerank(sc, args.alpha, args.epsilon)
        out["networkx"] = {"value": ne * it / tp, "unit": "edges/s", "cores": 1, "kind": "networkx",
                           "seconds": tp, "iterations": it,
                           "sample": f"nx.pagerank (networkx 3.4.2, tol=epsilon/N as nx defines it) to convergence "
                                     f"on RMAT-{sc} symmetric ({ne} stored edges, the largest sample kept within "
                                     f"the bench's time budget); nx.Graph build {tb:.1f}s excluded"}
    except Exception as e:  # noqa: BLE001
        out["networkx"] = {"error": repr(e)[:200]}
    return out


def networkx_cpu_legs(args):
    """The reference's NetworkX CPU path for BFS and Louvain on bounded R-MAT samples
    (same generator parameters, numpy twin), 1 core; NetworkX cannot hold the
    benchmark graphs, so the sample scale is stated."""
    import numpy as np
    from oracle import graph as og
    from oracle import rmat
    from oracle.baseline import networkx_bfs, networkx_louvain
    out = {}
    sb = 16
    s, d = rmat.rmat(sb, 16 << sb, seed=42)
    s, d, _ = og.symmetrize_dedup(s, d, None)
    root = int(s[0])
    tb, t, e_cc = networkx_bfs(s, d, root)
    out["bfs"] = {"value": (e_cc / t) / 1e6, "unit": "MTEPS", "cores": 1, "kind": "networkx",
                  "sample": f"nx.single_source_shortest_path_length, networkx 3.4.2, RMAT-{sb} symmetric "
                            f"({s.size} stored edges), 1 root; graph build {tb:.1f}s excluded"}
    sl = 14
    s, d = rmat.rmat(sl, 16 << sl, seed=42)
    w = rmat.rmat_weights(s.size, seed=43).astype(np.float64)
    s, d, w = og.symmetrize_dedup(s, d, w)
    tb, t, q = networkx_louvain(s, d, w)
    out["louvain"] = {"value": t, "unit": "s", "cores": 1, "kind": "networkx", "modularity": q,
                      "sample": f"nx.community.louvain_communities(seed=42) + modularity, networkx 3.4.2, "
                                f"RMAT-{sl} symmetric uniform weights ({s.size} stored edges); build {tb:.1f}s excluded"}
    return out


# ----------------------------------------------------------------------------- BFS
def ab_options(h, args):
    """--options name=value,...: handle options for A/B runs (include/cugraph_amd/ext.h)."""
    for kv in filter(None, (getattr(args, "options", "") or "").split(",")):
        k, v = kv.split("=")
        h.set_option(k, float(v))


def bfs_leg(p, args, child=False):
    import torch
    h = p.ResourceHandle(args.ctx.ptr if args.ctx else None)
    ab_options(h, args)
    scale = args.bfs_scale
    g, roots, deg = build_rmat_graph(p, h, scale, transposed=False, want_roots=args.bfs_roots, mg=args.mg)
    V, E = g.number_of_vertices(), g.number_of_edges()
    if deg is None:  # SG: degrees from the CSR (internal order == result order)
        off, _, _ = g.adjacency(h, transposed=False)
        deg_int = (off[1:] - off[:-1]).to(torch.int64)
    rates, stored, levels, bu, times, bytes_alg, spread = [], [], [], [], [], [], []
    number_map = None
    first_ms = None
    if not child:
        # first traversal on the fresh graph: the per-graph work (the bottom-up probe's
        # head table, the CSR's max degree) is inside it; module load was done by the
        # build's kernels and is not (the BFS kernels load with the library)
        src0 = torch.tensor([int(roots[0])] if args.rank == 0 else [], dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        barrier(args)
        t0 = time.perf_counter()
        p.bfs(h, g, src0, True, 0, True, False)
        torch.cuda.synchronize()
        first_ms = max_over_ranks(args, time.perf_counter() - t0) * 1e3
    for r in roots:
        mine = [int(r)] if args.rank == 0 else []
        src = torch.tensor(mine, dtype=torch.int32, device="cuda")
        if child:  # PMC pass: exactly one traversal per root
            p.bfs(h, g, src.clone(), True, 0, True, False)
            continue
        p.bfs(h, g, src.clone(), True, 0, True, False)  # warm
        samples, res = [], None
        for _ in range(args.bfs_reps):
            res = None  # the previous result's free (a device synchronize) stays off the clock
            s_in = src.clone()
            torch.cuda.synchronize()
            barrier(args)
            t0 = time.perf_counter()
            res = p.bfs(h, g, s_in, True, 0, True, False)
            torch.cuda.synchronize()
            barrier(args)
            samples.append(max_over_ranks(args, time.perf_counter() - t0))
        dist, pred, verts = res
        t = sorted(samples)[len(samples) // 2]  # median of the root's traversals
        reached = dist < 2**31 - 1
        # Graph500 TEPS: undirected edges of the source's component = stored directed edges / 2
        if deg is None:
            e_cc = int(deg_int[reached].sum().item())
            v_cc = int(reached.sum().item())
        else:
            e_cc = int(sum_over_ranks(args, float(deg[verts[reached].to(torch.int64)].sum().item())))
            v_cc = int(sum_over_ranks(args, float(reached.sum().item())))
        if number_map is None and deg is None:
            number_map = verts.cpu().numpy()  # internal id -> external id (SG)
        times.append(t)
        spread.append((min(samples), max(samples)))
        levels.append(h.last_bfs_levels())
        bu.append(h.last_bfs_bottom_up_steps())
        rates.append((e_cc / 2) / t / 1e6)
        stored.append(e_cc / t / 1e6)
        bytes_alg.append(4 * e_cc + 16 * v_cc)
    if child:
        return None
    hm = len(rates) / sum(1.0 / m for m in rates)
    hm_stored = len(stored) / sum(1.0 / m for m in stored)
    achieved = sum(bytes_alg) / sum(times) / 1e9 / args.world
    out = {"scale": scale, "vertices": V, "edges": E, "roots": len(rates),
           "mteps_harmonic_mean": hm, "mteps_min": min(rates), "mteps_max": max(rates),
           "stored_edge_mteps_harmonic_mean": hm_stored,
           "ms_mean": 1e3 * sum(times) / len(times), "ms_per_root_median": [round(1e3 * x, 4) for x in times],
           "ms_per_root_min_max": [[round(1e3 * a, 4), round(1e3 * b, 4)] for a, b in spread],
           "reps_per_root": args.bfs_reps,
           "timing": "median of reps_per_root timed traversals per root (after one warm traversal); MTEPS per root "
                     "from its median, harmonic mean over the roots",
           "levels": levels, "bottom_up_steps": bu,
           "first_call_ms": round(first_ms, 3),
           "first_call_note": "the first cugraph_bfs on the freshly built graph (from the first root; includes the "
                              "per-graph head table k_bfs_head); ms_per_root_median[0] is the same root's steady "
                              "traversal",
           "direction_optimizing": True, "n_gpus": args.world,
           "teps_counting": "Graph500: undirected edges of the source component / time (max over ranks)",
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                        "achieved_kind": "algorithmic-equivalent: the bytes a top-down pull over the source's "
                                         "component would read (4 E_cc + 16 V_cc, SURVEY.md §8d) / time; a "
                                         "direction-optimising traversal reads far fewer, so see frac_counter "
                                         "(counter bytes / time) for the memory system's actual load",
                        "algorithmic_bytes_per_launch": sum(bytes_alg) / len(bytes_alg) / args.world,
                        "ms_per_traversal": 1e3 * sum(times) / len(times),
                        "kernel": "one traversal (all levels, host wall time between synchronisations); "
                                  "bytes = 4 E_cc + 16 V_cc (SURVEY.md §8d), per rank at N > 1"}}
    if args.rank == 0 and args.world == 1 and not args.no_cpu_baseline:
        try:
            import numpy as np
            from oracle import cpu_native
            off, idx, _ = g.adjacency(h, transposed=False)
            off, idx = off.cpu().numpy().astype(np.int64), idx.cpu().numpy()
            # the first bench root, in internal ids
            root_int = int(np.nonzero(number_map == roots[0])[0][0])
            T = omp_threads()
            t1, d1, _ = cpu_native.bfs(off, idx, root_int, threads=1)
            tn, _, _ = cpu_native.bfs(off, idx, root_int, threads=T)
            e_cc = int((off[1:] - off[:-1])[d1 != np.iinfo(np.int32).max].sum())
            out["cpu_baseline_compiled"] = {
                "kind": "port", "source": "oracle/cpu_baseline.c (bfs_test.cpp:41-79 restated)",
                "single_thread": {"value": (e_cc / 2) / t1 / 1e6, "unit": "MTEPS", "cores": 1},
                "openmp": {"value": (e_cc / 2) / tn / 1e6, "unit": "MTEPS", "cores": T},
                "sample": f"one traversal from the first bench root on the same RMAT-{scale} graph (top-down)",
                "host": host_info(T)}
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline_compiled"] = {"error": repr(e)[:200]}
    return out


# ----------------------------------------------------------------------------- SSSP
SSSP_KERNELS = ("k_relax", "k_split", "k_sssp_", "k_pred_none", "k_weight_stats")


def sssp_leg(p, args, child=False):
    """SSSP (near-far, csrc/sssp.hip) on the BFS leg's graph with the bench's uniform
    [0, 1) fp32 weights (seed 43, cugraph_funcs.py:56-58; the reference benchmarks SSSP
    beside BFS, benchmarks/python_e2e/cugraph_funcs.py:122-123) from the first
    sssp_roots Graph500 roots, predecessors on; per source the median of bfs_reps timed
    calls.  TEPS counting as BFS (undirected edges of the source's component / time)."""
    import torch
    h = p.ResourceHandle(args.ctx.ptr if args.ctx else None)
    ab_options(h, args)
    scale = args.bfs_scale
    g, roots, _ = build_rmat_graph(p, h, scale, weighted=True, transposed=False, want_roots=args.bfs_roots)
    roots = roots[:args.sssp_roots]
    V, E = g.number_of_vertices(), g.number_of_edges()
    off, _, _ = g.adjacency(h, transposed=False)
    deg_int = (off[1:] - off[:-1]).to(torch.int64)
    del off
    times, rates, rounds, spread, bytes_alg, reached_n = [], [], [], [], [], []
    number_map = None
    first_ms = None
    for i, r in enumerate(roots):
        if child:
            p.sssp(h, g, int(r), float("inf"), True, False)
            continue
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = p.sssp(h, g, int(r), float("inf"), True, False)  # warm (the first: per-graph work inside)
        torch.cuda.synchronize()
        if i == 0:
            first_ms = (time.perf_counter() - t0) * 1e3
        samples = []
        for _ in range(args.bfs_reps):
            res = None
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = p.sssp(h, g, int(r), float("inf"), True, False)
            torch.cuda.synchronize()
            samples.append(time.perf_counter() - t0)
        verts, dist, _ = res
        if number_map is None:
            number_map = verts
        t = sorted(samples)[len(samples) // 2]
        reached = dist < torch.finfo(dist.dtype).max
        e_cc = int(deg_int[reached].sum().item())
        v_cc = int(reached.sum().item())
        times.append(t)
        spread.append((min(samples), max(samples)))
        rates.append((e_cc / 2) / t / 1e6)
        rounds.append(h.last_iterations())
        reached_n.append(v_cc)
        # algorithmic bytes: every reached vertex's adjacency (4 B index + 4 B weight per
        # edge) and offsets (8 B), its distance and predecessor (4 + 4 B)
        bytes_alg.append(8 * e_cc + 16 * v_cc)
        del res, verts, dist, reached
    if child:
        return None
    hm = len(rates) / sum(1.0 / m for m in rates)
    achieved = sum(bytes_alg) / sum(times) / 1e9
    out = {"scale": scale, "vertices": V, "edges": E, "weights": "uniform [0,1) fp32, seed 43", "roots": len(rates),
           "mteps_harmonic_mean": hm, "ms_mean": 1e3 * sum(times) / len(times),
           "ms_per_root_median": [round(1e3 * x, 4) for x in times],
           "ms_per_root_min_max": [[round(1e3 * a, 4), round(1e3 * b, 4)] for a, b in spread],
           "reps_per_root": args.bfs_reps, "rounds": rounds, "reached": reached_n,
           "first_call_ms": round(first_ms, 3), "predecessors": True,
           "teps_counting": "Graph500: undirected edges of the source component / time",
           "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                        "achieved_kind": "algorithmic-equivalent: 8 E_cc + 16 V_cc per traversal (each reached "
                                         "adjacency read once with its weights) / time",
                        "ms_per_traversal": 1e3 * sum(times) / len(times)}}
    if args.rank == 0 and args.world == 1 and not args.no_cpu_baseline:
        try:
            import numpy as np
            from oracle import cpu_native
            off, idx, w = g.adjacency(h, transposed=False)
            off, idx, w = off.cpu().numpy().astype(np.int64), idx.cpu().numpy(), w.cpu().numpy()
            nm = number_map.cpu().numpy()
            root_int = int(np.nonzero(nm == roots[0])[0][0])
            t1, d1, _, rr = cpu_native.sssp(off, idx, w, root_int)
            e_cc = int((off[1:] - off[:-1])[d1 < np.finfo(np.float32).max].sum())
            out["cpu_baseline"] = {
                "kind": "port", "source": "oracle/cpu_sssp.c (sssp_impl.cuh:79-270 near-far restated, fp32)",
                "value": (e_cc / 2) / t1 / 1e6, "unit": "MTEPS", "cores": 1, "seconds": t1, "rounds": rr,
                "sample": f"one traversal from the first root on the same RMAT-{scale} graph, predecessors "
                          "resolved after the timed loop",
                "host": host_info(1)}
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline"] = {"error": repr(e)[:200]}
    return out


def sssp_traffic(args):
    """HBM bytes per SSSP traversal (every SSSP kernel), 2 x FETCH_SIZE + WRITE_SIZE."""
    per = {}
    child = ["--traffic-child", "sssp", "--bfs-scale", str(args.bfs_scale), "--bfs-roots", str(args.bfs_roots),
             "--sssp-roots", str(args.sssp_roots)]
    n = args.sssp_roots
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = pmc_pass(ctr, child, SSSP_KERNELS)
        per[ctr] = sum(sum(v) for v in vals.values()) / n
    return (2.0 * per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024.0, per


# ----------------------------------------------------------------------------- Louvain
def louvain_leg(p, args, scale=None):
    """configs[4]: Louvain time-to-solution on a symmetrised R-MAT graph with uniform
    [0, 1) fp32 weights (seed 42, cugraph_funcs.py:56-58), max_level 100,
    resolution 1.0.  SG at N=1, the MG path (rows by source owner, RCCL) at N>1."""
    import torch
    h = p.ResourceHandle(args.ctx.ptr if args.ctx else None)
    ab_options(h, args)
    small, _, _ = build_rmat_graph(p, h, 10, weighted=True, transposed=False, mg=args.mg)
    p.louvain(h, small, 100, 1.0, False)  # module load + allocator warm-up off the clock
    del small
    scale = scale or args.louvain_scale
    free_gb = torch.cuda.mem_get_info()[0] / 2**30
    t0 = time.perf_counter()
    g, _, _ = build_rmat_graph(p, h, scale, weighted=True, transposed=False, mg=args.mg)
    build_s = time.perf_counter() - t0
    V, E = g.number_of_vertices(), g.number_of_edges()
    torch.cuda.synchronize()
    barrier(args)
    a0 = p.allocator_stats()
    t0 = time.perf_counter()
    _, _, q = p.louvain(h, g, 100, 1.0, False)
    torch.cuda.synchronize()
    barrier(args)
    t = max_over_ranks(args, time.perf_counter() - t0)
    a1 = p.allocator_stats()
    alloc = {"mallocs": a1["mallocs"] - a0["mallocs"], "malloc_s": round(a1["malloc_s"] - a0["malloc_s"], 4),
             "malloc_gib": round((a1["malloc_bytes"] - a0["malloc_bytes"]) / 2**30, 1),
             "oom_trims": a1["oom_trims"] - a0["oom_trims"]}
    sweep_bytes = max_over_ranks(args, h.last_louvain_sweep_bytes()) if args.world > 1 else 0.0
    return {"scale": scale, "vertices": V, "edges": E, "weights": "uniform [0,1) fp32, seed 43",
            "time_s": t, "modularity": q, "levels": h.last_louvain_levels(), "graph_build_s": round(build_s, 3),
            "sweep_bytes_per_rank_max": sweep_bytes, "device_free_gib_at_start": round(free_gb, 1),
            "allocator_during_call": alloc,
            "n_gpus": args.world,
            "path": "sg" if args.world == 1 else f"mg{args.world} ({'RCCL' if args.comm == 'rccl' else 'torch'})"}


# ----------------------------------------------------------------------------- main
def make_ctx(p, args, C):
    if args.comm == "rccl":
        return p.comms.init_rccl(C)
    return p.comms.init_torch(C)


def grid_name(args, C):
    return (f"2D {args.world // C}x{C} (rows x cols), "
            f"{'RCCL' if args.comm == 'rccl' else 'torch.distributed/gloo'}")


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_command(n, argv, port):
    """The torch.distributed.run command line of an N-rank run of this script."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """Start N ranks as a child process group (never exec: the parent has not
    touched the GPU, but a child keeps that true by construction); rank 0's JSON
    line reaches our stdout through the inherited descriptor."""
    cmd = launch_command(n, argv, free_port())
    log(f"[bench] launching {n} ranks: {' '.join(cmd[1:6])} ...")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=24, help="headline PageRank scale (BASELINE: RMAT-24 at every N)")
    ap.add_argument("--alpha", type=float, default=0.85)
    ap.add_argument("--epsilon", type=float, default=1e-6)
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--nx-pagerank-scale", type=int, default=17)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bfs", dest="bfs", action="store_true", default=True)
    ap.add_argument("--no-bfs", dest="bfs", action="store_false")
    ap.add_argument("--bfs-scale", type=int, default=24)
    ap.add_argument("--bfs-roots", type=int, default=8)
    ap.add_argument("--bfs-reps", type=int, default=5, help="timed traversals per root (median reported)")
    ap.add_argument("--sssp", dest="sssp", action="store_true", default=True)
    ap.add_argument("--no-sssp", dest="sssp", action="store_false")
    ap.add_argument("--sssp-roots", type=int, default=4, help="SSSP sources (the first BFS roots)")
    ap.add_argument("--no-rmat26", dest="rmat26", action="store_false", default=True,
                    help="skip the one-GPU RMAT-26 PageRank and Louvain legs (configs[3]/[4]'s graph)")
    ap.add_argument("--louvain", dest="louvain", action="store_true", default=True)
    ap.add_argument("--no-louvain", dest="louvain", action="store_false")
    ap.add_argument("--louvain-scale", type=int, default=None, help="default 23 + log2(N): RMAT-26 at 8 GPUs")
    ap.add_argument("--secondary", dest="secondary", action="store_true", default=True,
                    help="secondary PageRank legs: RMAT-22 at N=1, RMAT-26 at N=8, the other grid at N>1")
    ap.add_argument("--no-secondary", dest="secondary", action="store_false")
    ap.add_argument("--row-comm-size", type=int, default=None,
                    help="C of the R x C grid (default: the reference's rule, mg_utilities.cpp:60-63 -- the "
                         "largest divisor of N <= sqrt(N): 2 at N=8, R=4)")
    ap.add_argument("--comm", choices=["rccl", "torch"], default="rccl",
                    help="MG collectives: RCCL inside libcugraph_c (default), or torch.distributed callbacks "
                         "(code-path rehearsal with several ranks on one GPU; not a performance number)")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--traffic-child", choices=["pagerank", "bfs", "sssp"], default=None, help=argparse.SUPPRESS)
    ap.add_argument("--sssp-only", action="store_true", help="A/B aid: only the SSSP leg, its dict on stdout")
    ap.add_argument("--bfs-only", action="store_true", help="A/B aid: only the BFS leg, its dict on stdout")
    ap.add_argument("--louvain-only", action="store_true", help="A/B aid: only the Louvain leg, its dict on stdout")
    ap.add_argument("--options", default="", help="A/B aid: handle options name=value,... for the BFS / Louvain legs")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one command, N ranks (benchmarks/python_e2e/main.py:72-79 starts one worker
        # per GPU itself): run torch.distributed.run as a CHILD before anything here
        # touches the GPU, relay its output and exit code
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    grow = int(round(math.log2(max(world, 1))))
    if args.louvain_scale is None:
        args.louvain_scale = 23 + grow  # BASELINE configs[4]: RMAT-26 Louvain on 8 GPUs
    args.world, args.rank = world, rank
    args.mg = (rank, world) if world > 1 else None

    import torch
    import pylibcugraph as p

    args.ctx = None
    C = None
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("gloo")  # bootstrap + timing only; the data path is RCCL
        C = args.row_comm_size or p.comms.default_row_comm_size(world)
        args.ctx = make_ctx(p, args, C)
    torch.cuda.init()

    if args.traffic_child == "pagerank":
        pagerank_leg(p, args, args.scale, 1, 0)
        return
    if args.traffic_child == "bfs":
        bfs_leg(p, args, child=True)
        return
    if args.traffic_child == "sssp":
        sssp_leg(p, args, child=True)
        return
    if args.sssp_only:
        r = sssp_leg(p, args)
        log(f"[bench] sssp RMAT-{args.bfs_scale}: {r['mteps_harmonic_mean']:.1f} MTEPS, {r['ms_mean']:.3f} ms/traversal, "
            f"rounds {r['rounds']}")
        print(json.dumps(r), flush=True)
        return
    if args.bfs_only:
        r = bfs_leg(p, args)
        log(f"[bench] bfs RMAT-{args.bfs_scale}: {r['mteps_harmonic_mean']:.1f} MTEPS, {r['ms_mean']:.3f} ms/traversal")
        print(json.dumps(r), flush=True)
        return
    if args.louvain_only:
        r = louvain_leg(p, args)
        log(f"[bench] louvain RMAT-{r['scale']}: {r['time_s']:.3f}s Q={r['modularity']:.6f} levels={r['levels']}")
        print(json.dumps(r), flush=True)
        return

    r = pagerank_leg(p, args, args.scale, args.steps, args.warmup, args.ctx)
    out = {
        "metric": "PageRank edges/sec + BFS MTEPS on RMAT-24 at 1/2/4/8 MI355X",
        "value": r["value"],
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["t"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: device Graph500 R-MAT (a=.57 b=c=.19, ef 16, seed 42, scrambled), symmetrised+dedup",
        "config": {
            "workload": f"RMAT scale-{args.scale} PageRank fp32 (symmetric, unweighted), alpha {args.alpha}, "
                        f"epsilon {args.epsilon}",
            "model": "pagerank",
            "scale": args.scale,
            "vertices": r["V"],
            "edges": r["E"],
            "iterations_per_step": r["iters"][0] if r["iters"] else 0,
            "graph_build_s": round(r["build_s"], 3),
            "first_call_ms": round(r["first_ms"], 3),
            "next_graph_first_call_ms": round(r["next_graph_first_ms"], 3),
            "first_call_note": ("one cugraph_pagerank on the freshly built graph (out-weight sums, push schedule "
                                "build, calibration chunk, then the iterations to convergence), after "
                                "PageRank on RMAT-10 with each window size has loaded the code objects; "
                                "steady-state calls take "
                                f"ms_per_step; first call ran {r['first_iters']} iterations. "
                                "next_graph_first_call_ms: the same on a second fresh graph of this size after "
                                "the timed steps (the per-graph cost once the process has run one graph: no "
                                "first loads of the size's kernels, the allocator's blocks cached)"),
            "parallelism": "sg" if world == 1 else f"mg{world}: {grid_name(args, C)}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": ("k_pr_push16_w14 with the apply fused in (16K-destination windows from 2^23 vertices; below that k_pr_push16 + k_pr_apply; packed 16-bit entries; k_pr_push_q* for weighted graphs) = one PageRank iteration: HIP events on the library stream around "
                       "each chunk of iterations in the timed region / iterations run (inter-kernel gaps "
                       "included)" if world == 1 else
                       "one MG PageRank iteration per rank (row allgather + push + column reduce-scatter + apply + "
                       "allreduce, HIP events around all); bytes = this rank's 1/N share"),
            "achieved": r["achieved"],
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": r["achieved"] / HBM_PEAK_GBS,
            "traffic": None,
            "algorithmic_bytes_per_launch": r["bytes_per_iter"],
            "avg_kernel_ms": r["avg_ms"],
        },
    }
    if world > 1:  # MG comm bytes per rank and iteration (x~ allgather + u64 sums reduce-scatter)
        Rr = world // C
        out["roofline"]["comm_bytes_per_rank_iter"] = ((C - 1) * r["V"] / world * 4 + (Rr - 1) * r["V"] / world * 8)
    try:
        out["roofline"]["copy_ceiling_gbs"] = r["h"].measure_copy_bandwidth(4 << 30, 10)
    except Exception as e:  # noqa: BLE001
        out["roofline"]["copy_ceiling_gbs"] = f"unavailable: {e!r}"[:200]
    # (no nested profiler: a bench already running under rocprofv3 skips the traffic passes)
    under_prof = any(k.startswith("ROCPROF_") for k in os.environ)
    do_traffic = rank == 0 and world == 1 and not args.no_traffic and not under_prof
    # The PMC passes run in rocprofv3 child processes AFTER every timed leg: device memory
    # another process has freed is scrubbed by the driver when this process next maps it,
    # which made the RMAT-26 Louvain leg's 106 GB of hipMallocs take 0.60 s after the
    # children had run (2.84 vs 2.26 s), a cost no user call sees.
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = pagerank_cpu_baseline(p, r, args)
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline"] = {"error": repr(e)[:300]}
    mg_ref = None
    if world > 1:  # the default (K = 1) result, for the overlapped-chunk leg's bitwise check
        v1, x1 = p.pagerank(r["h"], r["g"], None, None, None, None, args.alpha, args.epsilon, 500, False)
        mg_ref = (v1.clone(), x1.view(torch.int32).clone(), r["h"].last_iterations())
        del v1, x1
    del r
    release_caches(p)

    if args.secondary:
        try:
            if world == 1:
                r2 = pagerank_leg(p, args, 22, args.steps, args.warmup)
                out["pagerank_rmat22"] = pagerank_summary(r2, args, "sg")
                del r2
                release_caches(p)
                # the reference Python path's graph: all-ones fp32 weights (simpleGraph.py:840-843),
                # detected at the first call and run on the unweighted push; then the same graph
                # on the entry-weight push (option pr_unit_w = 0: 32-bit entries + 4 B weights)
                for key, opts in (("pagerank_rmat24_weighted", None),
                                  ("pagerank_rmat24_weighted_entry_push", {"pr_unit_w": 0})):
                    r2 = pagerank_leg(p, args, args.scale, max(1, args.steps // 2), 1, weighted="ones",
                                      options=opts)
                    out[key] = pagerank_summary(r2, args, "sg")
                    out[key]["weights"] = "all-ones fp32 (cugraph.Graph unweighted edge list)"
                    out[key]["push"] = ("unweighted 16-bit entries (unit weights detected)" if opts is None else
                                        "32-bit entries + fp32 entry weights (option pr_unit_w = 0)")
                    del r2
                    release_caches(p)
                # configs[3]'s graph on one GPU: the single-GPU anchor of the 8-GPU run
                if args.rmat26:
                    r2 = pagerank_leg(p, args, 26, max(1, args.steps // 2), 1)
                    out["pagerank_rmat26"] = pagerank_summary(r2, args, "sg")
                    out["pagerank_rmat26"]["note"] = "configs[3]'s graph (RMAT-26) on one GPU"
                    del r2
                    release_caches(p)
            else:
                alt = p.comms.flat_row_comm_size(world) if C != p.comms.flat_row_comm_size(world) \
                    else p.comms.default_row_comm_size(world)
                if alt != C:
                    ctx2 = make_ctx(p, args, alt)
                    r2 = pagerank_leg(p, args, args.scale, args.steps, args.warmup, ctx2)
                    out["pagerank_alt_grid"] = pagerank_summary(r2, args, grid_name(args, alt))
                    del r2
                    release_caches(p)
                    barrier(args)
                    ctx2.free()
                if world // C > 1 and mg_ref is not None:
                    out["pagerank_overlap_k4"] = overlap_leg(p, args, mg_ref, C)
                    release_caches(p)
                if world == 8:
                    r2 = pagerank_leg(p, args, 26, max(1, args.steps // 2), 1, args.ctx)
                    out["pagerank_rmat26"] = pagerank_summary(r2, args, grid_name(args, C))
                    del r2
        except Exception as e:  # noqa: BLE001
            out["secondary_error"] = repr(e)[:300]
        release_caches(p)
    if args.bfs:
        try:
            out["bfs"] = bfs_leg(p, args)
            log(f"[bench] bfs RMAT-{args.bfs_scale}: {out['bfs']['mteps_harmonic_mean']:.1f} MTEPS, "
                f"{out['bfs']['ms_mean']:.3f} ms/traversal")
        except Exception as e:  # noqa: BLE001
            out["bfs"] = {"status": "failed", "error": repr(e)[:300]}
        release_caches(p)
    if args.sssp and world == 1:
        try:
            out["sssp"] = sssp_leg(p, args)
            log(f"[bench] sssp RMAT-{args.bfs_scale}: {out['sssp']['mteps_harmonic_mean']:.1f} MTEPS, "
                f"{out['sssp']['ms_mean']:.3f} ms/traversal, rounds {out['sssp']['rounds']}")
        except Exception as e:  # noqa: BLE001
            out["sssp"] = {"status": "failed", "error": repr(e)[:300]}
        release_caches(p)
    if args.louvain:
        try:
            out["louvain"] = louvain_leg(p, args)
            log(f"[bench] louvain: RMAT-{out['louvain']['scale']} {out['louvain']['time_s']:.3f}s "
                f"Q={out['louvain']['modularity']:.6f} levels={out['louvain']['levels']}")
        except Exception as e:  # noqa: BLE001
            out["louvain"] = {"status": "failed", "error": repr(e)[:300]}
    if args.louvain and args.rmat26 and world == 1:
        try:  # configs[4]'s graph on one GPU (SG Louvain RMAT-26)
            release_caches(p)
            out["louvain_rmat26"] = louvain_leg(p, args, 26)
            out["louvain_rmat26"]["note"] = "configs[4]'s graph (RMAT-26, uniform weights) on one GPU"
            log(f"[bench] louvain: RMAT-26 {out['louvain_rmat26']['time_s']:.3f}s "
                f"Q={out['louvain_rmat26']['modularity']:.6f} levels={out['louvain_rmat26']['levels']}")
        except Exception as e:  # noqa: BLE001
            out["louvain_rmat26"] = {"status": "failed", "error": repr(e)[:300]}
    if do_traffic:
        release_caches(p)
        try:
            tb, detail = pagerank_traffic(args)
            out["roofline"]["traffic"] = tb
            out["roofline"]["traffic_note"] = (
                "HBM bytes per iteration (k_pr_push [+ k_pr_apply when not fused]) = 2 x FETCH_SIZE + WRITE_SIZE (KiB) from separate "
                f"rocprofv3 --pmc passes: {detail}")
        except Exception as e:  # noqa: BLE001
            out["roofline"]["traffic_note"] = f"unavailable: {e!r}"[:300]
        if isinstance(out.get("bfs"), dict) and "roofline" in out["bfs"]:
            try:
                tb, detail = bfs_traffic(args, args.bfs_roots)
                out["bfs"]["roofline"]["traffic"] = tb
                ms_t = out["bfs"]["roofline"]["ms_per_traversal"]
                out["bfs"]["roofline"]["achieved_counter"] = tb / (ms_t * 1e-3) / 1e9
                out["bfs"]["roofline"]["frac_counter"] = tb / (ms_t * 1e-3) / 1e9 / HBM_PEAK_GBS
                out["bfs"]["roofline"]["traffic_note"] = (
                    "HBM bytes per traversal (every BFS kernel but the per-graph head table k_bfs_head, "
                    "reported as per_graph_kib) = 2 x FETCH_SIZE + WRITE_SIZE (KiB) from separate rocprofv3 "
                    f"--pmc passes over one traversal per root: {detail}")
            except Exception as e:  # noqa: BLE001
                out["bfs"]["roofline"]["traffic_note"] = f"unavailable: {e!r}"[:300]
        if isinstance(out.get("sssp"), dict) and "roofline" in out["sssp"]:
            try:
                tb, detail = sssp_traffic(args)
                out["sssp"]["roofline"]["traffic"] = tb
                ms_t = out["sssp"]["roofline"]["ms_per_traversal"]
                out["sssp"]["roofline"]["frac_counter"] = tb / (ms_t * 1e-3) / 1e9 / HBM_PEAK_GBS
                out["sssp"]["roofline"]["traffic_note"] = (
                    "HBM bytes per traversal (every SSSP kernel) = 2 x FETCH_SIZE + WRITE_SIZE (KiB) from "
                    f"separate rocprofv3 --pmc passes over one traversal per root: {detail}")
            except Exception as e:  # noqa: BLE001
                out["sssp"]["roofline"]["traffic_note"] = f"unavailable: {e!r}"[:300]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            nxb = networkx_cpu_legs(args)
            if isinstance(out.get("bfs"), dict) and "mteps_harmonic_mean" in out["bfs"]:
                out["bfs"]["cpu_baseline"] = nxb["bfs"]
            if isinstance(out.get("louvain"), dict) and "time_s" in out["louvain"]:
                out["louvain"]["cpu_baseline"] = nxb["louvain"]
        except Exception as e:  # noqa: BLE001
            log(f"[bench] networkx baselines unavailable: {e!r}")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        args.ctx.free()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

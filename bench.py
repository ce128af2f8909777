#!/usr/bin/env python3
"""Benchmark: PageRank edges/s (+ BFS MTEPS) on Graph500 R-MAT, MI355X.

BASELINE.json metric: "PageRank edges/sec + BFS MTEPS on RMAT-24 at 1/2/4/8 MI355X".
Workload at N=1 (configs[1]): RMAT scale-22, symmetrised + deduplicated,
unweighted, fp32 PageRank, alpha 0.85, epsilon 1e-6.  A "step" is one complete
``cugraph_pagerank`` call (power iteration to convergence) on the resident graph.
value = stored edges x PageRank iterations x steps / timed seconds (whole job).

Extra fields on the same JSON line:
  roofline      -- the PageRank iteration kernels: algorithmic bytes/iteration
                   (4E + 16V) / average iteration time from HIP events recorded
                   around each 16-iteration chunk on the library's stream during
                   the timed region (divided by the iterations run); peak 8 TB/s
                   (MI355X_MICROARCH.md).
  cpu_baseline  -- NetworkX's PageRank loop (scipy CSR, fp64, 1 core;
                   oracle/baseline.py) for a few iterations on the SAME graph.
  bfs           -- configs[2]: RMAT scale-24 BFS MTEPS (Graph500 counting), when
                   the BFS path is available.
  louvain       -- configs[4]: Louvain time-to-solution, modularity and levels on
                   RMAT scale 23 + log2(N) (scale 26 at 8 GPUs), uniform weights.
  bfs.cpu_baseline / louvain.cpu_baseline -- the reference's NetworkX CPU path
                   (nx.single_source_shortest_path_length, nx louvain_communities)
                   on bounded R-MAT samples (RMAT-16 / RMAT-14; NetworkX cannot
                   hold the benchmark graphs), N=1 only.

Multi-GPU (--gpus N, launched by torch.distributed.run, one process per GPU):
weak scaling, R-MAT scale 22 + log2(N) for PageRank (the headline value); the
BFS leg stays on RMAT-24 at every N as BASELINE.json names it.  Every rank generates
and deduplicates the same edge list, keeps its 1/N slice, and the MG graph is
built collectively (cugraph_mg_graph_create: hash owners, degree renumbering, 2D
R x C edge blocks); PageRank and BFS then run over RCCL communicators created
inside libcugraph_c (pylibcugraph.comms.init_rccl).  torch.distributed (gloo)
is only used for the RCCL unique id, the timing barrier and the max over ranks.
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


def release_caches(p):
    """Between legs: torch's cached blocks and libcugraph_c's caching allocator."""
    import torch
    torch.cuda.synchronize()
    p.trim_device_cache()
    torch.cuda.empty_cache()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_rmat_graph(p, h, scale, seed=42, weighted=False, transposed=True, want_roots=0, mg=None):
    """Device R-MAT -> symmetrise + dedup (cugraph.Graph preprocessing) -> graph.
    mg = (rank, world): every rank makes the same edge list and passes its slice to
    the collective MGGraph build."""
    import numpy as np
    import torch
    n = 16 << scale
    s, d = p.generators.generate_rmat_edgelist(h, scale, n, 0.57, 0.19, 0.19, seed, False, True)
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
        sl = slice(lo, hi)
        g = p.MGGraph(h, props, s[sl].contiguous(), d[sl].contiguous(), None if w is None else w[sl].contiguous(),
                      store_transposed=transposed, num_edges=E)
    del s, d, w
    torch.cuda.synchronize()
    return g, roots, deg


def pagerank_leg(p, args):
    import torch
    h = p.ResourceHandle(args.ctx.ptr if args.ctx else None)
    t0 = time.perf_counter()
    g, _, _ = build_rmat_graph(p, h, args.scale, mg=args.mg)
    build_s = time.perf_counter() - t0
    V, E = g.number_of_vertices(), g.number_of_edges()
    log(f"[bench] RMAT-{args.scale}: V={V} E={E} (build {build_s:.2f}s)")
    for _ in range(args.warmup):
        p.pagerank(h, g, None, None, None, None, args.alpha, args.epsilon, 500, False)
    torch.cuda.synchronize()
    times, iters, kms, klaunch = [], [], 0.0, 0
    h.set_profiling(True)
    barrier(args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        p.pagerank(h, g, None, None, None, None, args.alpha, args.epsilon, 500, False)
        iters.append(h.last_iterations())
        kms += h.last_hot_kernel_ms()
        klaunch += h.last_hot_kernel_launches()
    torch.cuda.synchronize()
    barrier(args)
    t = time.perf_counter() - t0
    h.set_profiling(False)
    it_total = sum(iters)
    value = E * it_total / t
    # algorithmic bytes of one rank's share: 4E/N + 16V/N
    bytes_per_iter = (4 * E + 16 * V) / args.world
    avg_ms = kms / max(klaunch, 1)
    achieved = bytes_per_iter / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    return dict(h=h, g=g, V=V, E=E, t=t, iters=iters, value=value, avg_ms=avg_ms, achieved=achieved,
                bytes_per_iter=bytes_per_iter, build_s=build_s)


def cpu_baseline_leg(p, r, args):
    from oracle.baseline import pagerank_scipy_iterations
    off, idx, _ = r["g"].adjacency(r["h"], transposed=True)
    off, idx = off.cpu().numpy(), idx.cpu().numpy()
    t, eps = pagerank_scipy_iterations(off, idx, r["V"], iterations=args.cpu_iters)
    return {"value": eps, "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": f"{args.cpu_iters} NetworkX-style scipy power iterations (fp64, 1 thread) on the same "
                      f"RMAT-{args.scale} graph ({t:.1f}s); graph build excluded as on the GPU"}


def traffic_leg(args):
    """HBM bytes per PageRank iteration from PMC counters: a child process runs the
    PageRank leg under ``rocprofv3 --pmc`` once per counter (FETCH_SIZE and
    WRITE_SIZE cannot share a pass), MI355X_MICROARCH.md "HBM": bytes = 2 x
    FETCH_SIZE (gfx950 tallies 128-B requests at 64 B) + WRITE_SIZE, both in KiB.
    Launches after convergence (no-ops) are skipped."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    per_iter = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory(dir="/tmp") as d:
            cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
                   sys.executable, os.path.abspath(__file__), "--traffic-child", "--scale", str(args.scale),
                   "--steps", "1", "--warmup", "0", "--no-bfs", "--no-cpu-baseline"]
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                               timeout=300)
            if r.returncode != 0:
                return None, f"rocprofv3 {ctr} rc={r.returncode}: {r.stderr.decode()[-300:]}"
            rows = []
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                rows += list(csv.DictReader(open(f)))
        tot = 0.0
        for kern in ("k_pr_push", "k_pr_apply"):
            vals = [float(x["Counter_Value"]) for x in rows if kern in x["Kernel_Name"]]
            if not vals and kern == "k_pr_apply":
                continue  # fused apply (default): the push kernel does it
            if not vals:
                return None, f"no {kern} launches under rocprofv3"
            live = [v for v in vals if v > 0.01 * max(vals)]
            tot += sum(live) / len(live)
        per_iter[ctr] = tot
    return (2.0 * per_iter["FETCH_SIZE"] + per_iter["WRITE_SIZE"]) * 1024.0, per_iter


def bfs_leg(p, args):
    import torch
    h = p.ResourceHandle(args.ctx.ptr if args.ctx else None)
    scale = args.bfs_scale
    g, roots, deg = build_rmat_graph(p, h, scale, transposed=False, want_roots=args.bfs_roots, mg=args.mg)
    V, E = g.number_of_vertices(), g.number_of_edges()
    if deg is None:  # SG: degrees from the CSR (internal order == result order)
        off, _, _ = g.adjacency(h, transposed=False)
        deg_int = (off[1:] - off[:-1]).to(torch.int64)
    rates, stored, levels, bu, times = [], [], [], [], []
    for r in roots:
        mine = [int(r)] if args.rank == 0 else []
        src = torch.tensor(mine, dtype=torch.int32, device="cuda")
        p.bfs(h, g, src.clone(), True, 0, True, False)  # warm
        torch.cuda.synchronize()
        barrier(args)
        t0 = time.perf_counter()
        dist, pred, verts = p.bfs(h, g, src.clone(), True, 0, True, False)
        torch.cuda.synchronize()
        barrier(args)
        t = max_over_ranks(args, time.perf_counter() - t0)
        reached = dist < 2**31 - 1
        # Graph500 TEPS: undirected edges of the source's component = stored directed edges / 2
        if deg is None:
            e_cc = int(deg_int[reached].sum().item())
        else:
            e_cc = int(sum_over_ranks(args, float(deg[verts[reached].to(torch.int64)].sum().item())))
        times.append(t)
        levels.append(h.last_bfs_levels())
        bu.append(h.last_bfs_bottom_up_steps())
        rates.append((e_cc / 2) / t / 1e6)
        stored.append(e_cc / t / 1e6)
    hm = len(rates) / sum(1.0 / m for m in rates)
    hm_stored = len(stored) / sum(1.0 / m for m in stored)
    return {"scale": scale, "vertices": V, "edges": E, "roots": len(rates),
            "mteps_harmonic_mean": hm, "mteps_min": min(rates), "mteps_max": max(rates),
            "stored_edge_mteps_harmonic_mean": hm_stored,
            "ms_mean": 1e3 * sum(times) / len(times), "levels": levels, "bottom_up_steps": bu,
            "direction_optimizing": True, "n_gpus": args.world,
            "teps_counting": "Graph500: undirected edges of the source component / time (max over ranks)"}


def louvain_leg(p, args):
    """configs[4]: Louvain time-to-solution on a symmetrised R-MAT graph with uniform
    [0, 1) fp32 weights (seed 42, cugraph_funcs.py:56-58), max_level 100,
    resolution 1.0.  SG at N=1, the MG path (rows by source owner, RCCL) at N>1."""
    import torch
    h = p.ResourceHandle(args.ctx.ptr if args.ctx else None)
    small, _, _ = build_rmat_graph(p, h, 10, weighted=True, transposed=False, mg=args.mg)
    p.louvain(h, small, 100, 1.0, False)  # module load + allocator warm-up off the clock
    del small
    scale = args.louvain_scale
    t0 = time.perf_counter()
    g, _, _ = build_rmat_graph(p, h, scale, weighted=True, transposed=False, mg=args.mg)
    build_s = time.perf_counter() - t0
    V, E = g.number_of_vertices(), g.number_of_edges()
    torch.cuda.synchronize()
    barrier(args)
    t0 = time.perf_counter()
    _, _, q = p.louvain(h, g, 100, 1.0, False)
    torch.cuda.synchronize()
    barrier(args)
    t = max_over_ranks(args, time.perf_counter() - t0)
    return {"scale": scale, "vertices": V, "edges": E, "weights": "uniform [0,1) fp32, seed 43",
            "time_s": t, "modularity": q, "levels": h.last_louvain_levels(), "graph_build_s": round(build_s, 3),
            "n_gpus": args.world,
            "path": "sg" if args.world == 1 else f"mg{args.world} ({'RCCL' if args.comm == 'rccl' else 'torch'})"}


def cpu_networkx_legs(args):
    """the reference's NetworkX CPU path for BFS and Louvain, on bounded
    R-MAT samples (same generator parameters, numpy twin), 1 core.  NetworkX's
    dict-of-dicts graph cannot hold RMAT-23/24, so the sample scale is stated."""
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


def stream_copy_gbs(nbytes=4 << 30, reps=10):
    """Measured HBM ceiling: device-to-device copy of a 4 GiB buffer,
    read + write bytes / time, HIP events."""
    import torch
    a = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda")
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return gbs


def barrier(args):
    if args.world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(args, t):
    if args.world == 1:
        return t
    import torch
    import torch.distributed as dist
    x = torch.tensor([t], dtype=torch.float64)
    dist.all_reduce(x, op=dist.ReduceOp.MAX)
    return float(x[0])


def sum_over_ranks(args, v):
    if args.world == 1:
        return v
    import torch
    import torch.distributed as dist
    x = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(x)
    return float(x[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scale", type=int, default=None)
    ap.add_argument("--alpha", type=float, default=0.85)
    ap.add_argument("--epsilon", type=float, default=1e-6)
    ap.add_argument("--cpu-iters", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bfs", dest="bfs", action="store_true", default=True)
    ap.add_argument("--no-bfs", dest="bfs", action="store_false")
    ap.add_argument("--bfs-scale", type=int, default=None)
    ap.add_argument("--louvain", dest="louvain", action="store_true", default=True)
    ap.add_argument("--no-louvain", dest="louvain", action="store_false")
    ap.add_argument("--louvain-scale", type=int, default=None, help="default 23 + log2(N): RMAT-26 at 8 GPUs")
    ap.add_argument("--row-comm-size", type=int, default=None, help="C of the R x C grid (default: R <= C)")
    ap.add_argument("--comm", choices=["rccl", "torch"], default="rccl",
                    help="MG collectives: RCCL inside libcugraph_c (default), or torch.distributed callbacks "
                         "(code-path rehearsal with several ranks on one GPU; not a performance number)")
    ap.add_argument("--bfs-roots", type=int, default=8)
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--traffic-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    grow = int(round(math.log2(max(world, 1))))
    if args.scale is None:
        args.scale = 22 + grow
    if args.bfs_scale is None:
        args.bfs_scale = 24  # BASELINE: BFS on RMAT-24 at 1/2/4/8 GPUs (fixed graph)
    if args.louvain_scale is None:
        args.louvain_scale = 23 + grow  # BASELINE configs[4]: RMAT-26 Louvain on 8 GPUs
    args.world, args.rank = world, rank
    args.mg = (rank, world) if world > 1 else None

    import torch
    import pylibcugraph as p

    args.ctx = None
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group("gloo")  # bootstrap + timing only; the data path is RCCL
        if args.comm == "rccl":
            args.ctx = p.comms.init_rccl(args.row_comm_size)
        else:
            args.ctx = p.comms.init_torch(args.row_comm_size)
    torch.cuda.init()

    r = pagerank_leg(p, args)
    if args.traffic_child:
        return
    r["t"] = max_over_ranks(args, r["t"])
    r["value"] = r["E"] * sum(r["iters"]) / r["t"]
    log(f"[bench] pagerank: {r['value']:.4g} edges/s, iters {r['iters']}, kernel {r['avg_ms']:.4f} ms/iter, "
        f"{r['achieved']:.1f} GB/s algorithmic")
    grid = None
    if world > 1:
        C = args.ctx.row_comm_size
        grid = f"2D {world // C}x{C} (rows x cols), {'RCCL' if args.comm == 'rccl' else 'torch.distributed/gloo'}"

    out = {
        "metric": "PageRank edges/sec + BFS MTEPS on RMAT-24 at 1/2/4/8 MI355X",
        "value": r["value"],
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["t"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
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
            "parallelism": "sg" if world == 1 else f"mg{world}: {grid}",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": ("k_pr_push_q + k_pr_apply (one PageRank iteration): HIP events around each 16-iteration chunk on the "
                       "library stream / iterations run (inter-kernel gaps and post-convergence no-op launches included)" if world == 1 else
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
        C = args.ctx.row_comm_size
        Rr = world // C
        out["roofline"]["comm_bytes_per_rank_iter"] = ((C - 1) * r["V"] / world * 4 + (Rr - 1) * r["V"] / world * 8)
    try:
        out["roofline"]["stream_copy_gbs"] = stream_copy_gbs()
    except Exception as e:  # noqa: BLE001
        out["roofline"]["stream_copy_gbs"] = f"unavailable: {e!r}"[:200]
    # (no nested profiler: a bench already running under rocprofv3 skips the traffic passes)
    under_prof = any(k.startswith("ROCPROF_") for k in os.environ)
    if rank == 0 and world == 1 and not args.no_traffic and not under_prof:
        try:
            tb, detail = traffic_leg(args)
            out["roofline"]["traffic"] = tb
            out["roofline"]["traffic_note"] = (
                "HBM bytes per iteration (k_pr_push + k_pr_apply) = 2 x FETCH_SIZE + WRITE_SIZE from separate "
                f"rocprofv3 --pmc passes: {detail}" if tb else f"unavailable: {detail}")
        except Exception as e:  # noqa: BLE001
            out["roofline"]["traffic_note"] = f"unavailable: {e!r}"[:300]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline_leg(p, r, args)
        except Exception as e:  # noqa: BLE001
            out["cpu_baseline"] = {"error": repr(e)}
    if args.bfs:
        try:
            del r
            release_caches(p)
            out["bfs"] = bfs_leg(p, args)
        except Exception as e:  # noqa: BLE001
            out["bfs"] = {"status": "failed", "error": repr(e)[:300]}
    if args.louvain:
        try:
            release_caches(p)
            out["louvain"] = louvain_leg(p, args)
            log(f"[bench] louvain: RMAT-{out['louvain']['scale']} {out['louvain']['time_s']:.3f}s "
                f"Q={out['louvain']['modularity']:.6f} levels={out['louvain']['levels']}")
        except Exception as e:  # noqa: BLE001
            out["louvain"] = {"status": "failed", "error": repr(e)[:300]}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            nxb = cpu_networkx_legs(args)
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
        r = None
        args.ctx.free()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

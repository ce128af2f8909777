"""One-rank RCCL MG PageRank against single-GPU PageRank on the same graph (measurement
and diagnosis aid, not product).

usage: python scripts/mg_one_rank.py [SCALE] [VARIANT ...]
One process, torch.distributed world of 1, the library's RCCL communicators
(pylibcugraph.comms.init_rccl(1)): the MG path's every step -- x~ allgather, push,
apply or fused apply, u64 allreduce, state kernel -- runs through RCCL with one rank.
Prints ms per iteration (HIP events on the library stream, 16-iteration calls) for SG
and MG and their ratio; then, per VARIANT (handle options NAME=VALUE joined by ',',
"-" = the defaults), the MG converged result against SG's: iterations,
bit equality, worst relative error and the degrees of the vertices that differ.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def timed(p, h, g, calls=5):
    def run():
        try:
            p.pagerank(h, g, None, None, None, None, 0.85, 0.0, 16, False)
        except RuntimeError as e:
            if "converge" not in str(e):
                raise
    for _ in range(2):
        run()
    h.set_profiling(True)
    ms, n = 0.0, 0
    for _ in range(calls):
        run()
        ms += h.last_hot_kernel_ms()
        n += h.last_hot_kernel_launches()
    h.set_profiling(False)
    return ms / max(n, 1)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    import pylibcugraph as p
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    variants = sys.argv[2:] or ["-"]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(bench.free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    torch.cuda.set_device(0)
    h = p.ResourceHandle()
    g, _, _ = bench.build_rmat_graph(p, h, scale, transposed=True)
    sg_ms = timed(p, h, g)
    v, x = p.pagerank(h, g, None, None, None, None, 0.85, 1e-6, 500, False)
    it_sg = h.last_iterations()
    off, _, _ = g.adjacency(h, transposed=True)
    ext = v.cpu().numpy().astype(np.int64)
    n_ext = int(ext.max()) + 1
    sg_x = np.zeros(n_ext, np.float32)
    sg_x[ext] = x.cpu().numpy()
    deg = np.zeros(n_ext, np.int64)
    deg[ext] = (off[1:] - off[:-1]).cpu().numpy()
    del off
    root = int(ext[0])  # the largest-degree vertex
    sg_dist = None
    try:
        dv, _, vv = p.bfs(h, g, np.asarray([root], np.int32), True, 0, True, False)
        sg_dist = np.full(n_ext, -2, np.int64)
        sg_dist[vv.cpu().numpy().astype(np.int64)] = dv.cpu().numpy()
    except RuntimeError as e:
        print(f"  SG BFS: {e}", flush=True)
    if os.environ.get("SG_PACKED0"):  # the 32-bit-entry push on a second SG graph
        h.set_option("pr_packed", 0)
        g2, _, _ = bench.build_rmat_graph(p, h, scale, transposed=True)
        v2, x2 = p.pagerank(h, g2, None, None, None, None, 0.85, 1e-6, 500, False)
        h.set_option("pr_packed", 1)
        r2 = sg_x[v2.cpu().numpy().astype(np.int64)]
        print(f"  SG 32-bit entries: iterations {h.last_iterations()}, bitwise equal "
              f"{bool(np.array_equal(x2.cpu().numpy().view(np.int32), r2.view(np.int32)))}", flush=True)
        g2 = None
    g = None
    p.trim_device_cache()
    ctx = p.comms.init_rccl(1)
    hm = p.ResourceHandle(ctx.ptr)
    gm, _, _ = bench.build_rmat_graph(p, hm, scale, transposed=True, mg=(0, 1))
    print(f"  graphs: SG V={len(ext)} E={int(deg.sum())}; MG V={gm.number_of_vertices()} E={gm.number_of_edges()}",
          flush=True)
    try:
        dm, _, vm0 = p.bfs(hm, gm, np.asarray([root], np.int32), True, 0, True, False)
        ids0 = vm0.cpu().numpy().astype(np.int64)
        if sg_dist is not None:
            print(f"  BFS from {root}: MG distances equal SG {bool(np.array_equal(dm.cpu().numpy(), sg_dist[ids0]))}",
                  flush=True)
    except RuntimeError as e:
        print(f"  MG BFS: {e}", flush=True)
    mg_ms = timed(p, hm, gm)
    print(f"RMAT-{scale}: SG {sg_ms:.4f} ms/iteration, 1-rank RCCL MG {mg_ms:.4f} ms/iteration "
          f"(ratio {mg_ms / sg_ms:.3f}); SG iterations {it_sg}", flush=True)
    for var in variants:
        opts = [] if var == "-" else [kv.split("=", 1) for kv in var.split(",")]
        for k, val in opts:
            hm.set_option(k, float(val))
        vm, xm = p.pagerank(hm, gm, None, None, None, None, 0.85, 1e-6, 500, False)
        it_mg = hm.last_iterations()
        hm.set_option(None, 0)
        ids = vm.cpu().numpy().astype(np.int64)
        mx = xm.cpu().numpy()
        ref = sg_x[ids]
        same = bool(np.array_equal(mx.view(np.int32), ref.view(np.int32)))
        rel = np.abs(mx.astype(np.float64) - ref) / np.maximum(np.abs(ref.astype(np.float64)), 1e-30)
        bad = rel > 1e-3
        dq = np.quantile(deg[ids[bad]], [0, 0.5, 0.99, 1]).tolist() if bad.any() else []
        print(f"  [{var}] MG iterations {it_mg}; bitwise equal {same}; sum {float(mx.astype(np.float64).sum()):.6f}; "
              f"max rel err {float(rel.max()):.3e}; {int(bad.sum())} vertices off > 1e-3 "
              f"(degree quantiles 0/.5/.99/1 {dq}; all vertices {np.quantile(deg[ids], [0, 0.5, 0.99, 1]).tolist()})",
              flush=True)
    gm = None
    hm = None
    ctx.free()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

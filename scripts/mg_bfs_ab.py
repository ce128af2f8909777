"""Multi-GPU BFS direction thresholds on one rank (measurement aid, not product).

usage: mg_bfs_ab.py SCALE ALPHA,BETA[,PIPELINED] [...]
The MG BFS code path (2D top-down, 1D bottom-up, csrc/mg_bfs.hip) through a one-rank
RCCL communicator on the bench's R-MAT graph: ms per traversal (median of 5) from the
bench's 8 roots for each (mg_bfs_alpha, mg_bfs_beta), with the single-GPU BFS beside it.
One rank has no communication, so this prices the kernels' top-down / bottom-up trade
only; a multi-rank run adds the exchanges (row allgather + column all-to-all top-down,
a V/8-byte bitmap allgather bottom-up).
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def time_roots(p, h, g, roots, reps=5):
    import torch
    per = []
    for r in roots:
        src = torch.tensor([r], dtype=torch.int32, device="cuda")
        p.bfs(h, g, src.clone(), True, 0, True, False)  # warm
        ts = []
        for _ in range(reps):
            s_in = src.clone()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = p.bfs(h, g, s_in, True, 0, True, False)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del res
        per.append(statistics.median(ts) * 1e3)
    return per


def main():
    import torch
    import torch.distributed as dist
    import bench
    import pylibcugraph as p
    scale = int(sys.argv[1])
    settings = [tuple(float(x) for x in a.split(",")) for a in sys.argv[2:]]
    h = p.ResourceHandle()
    g, roots, _ = bench.build_rmat_graph(p, h, scale, transposed=False, want_roots=8)
    roots = [int(x) for x in roots]
    sg = time_roots(p, h, g, roots)
    print(f"SG: mean {statistics.mean(sg):.3f} ms/traversal, per root {[round(x, 3) for x in sg]}", flush=True)
    g = None
    p.trim_device_cache()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(bench.free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    ctx = p.comms.init_rccl(1)
    try:
        hm = p.ResourceHandle(ctx.ptr)
        gm, _, _ = bench.build_rmat_graph(p, hm, scale, transposed=False, mg=(0, 1))
        for st in settings:
            a, b = st[0], st[1]
            pipe = int(st[2]) if len(st) > 2 else 1
            hm.set_option("mg_bfs_alpha", a)
            hm.set_option("mg_bfs_beta", b)
            hm.set_option("mg_bfs_pipelined", pipe)
            t = time_roots(p, hm, gm, roots)
            print(f"MG one rank alpha {a:g} beta {b:g} pipelined {pipe}: mean {statistics.mean(t):.3f} ms/traversal, "
                  f"per root {[round(x, 3) for x in t]}", flush=True)
        gm = None
        hm = None
        torch.cuda.synchronize()
        p.trim_device_cache()
    finally:
        ctx.free()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

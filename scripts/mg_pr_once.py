"""One-rank RCCL MG PageRank and Louvain with wall times (for a kernel trace;
measurement aid, not product).  usage: mg_pr_once.py SCALE"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    import bench
    import pylibcugraph as p
    scale = int(sys.argv[1])
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(bench.free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    ctx = p.comms.init_rccl(1)

    def timed(what, f):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = f()
        torch.cuda.synchronize()
        print(f"{what}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
        return r

    try:
        hm = p.ResourceHandle(ctx.ptr)
        gm, _, _ = timed("MG build (unweighted)", lambda: bench.build_rmat_graph(p, hm, scale, transposed=True, mg=(0, 1)))
        for i in range(3):
            timed(f"MG pagerank call {i}", lambda: p.pagerank(hm, gm, None, None, None, None, 0.85, 1e-6, 500, False))
        gm = None
        p.trim_device_cache()
        gw, _, _ = timed("MG build (weighted)", lambda: bench.build_rmat_graph(p, hm, scale, weighted=True,
                                                                             transposed=False, mg=(0, 1)))
        for i in range(2):
            timed(f"MG louvain call {i}", lambda: p.louvain(hm, gw, 100, 1.0, False))
        gw = None
        hm = None
        torch.cuda.synchronize()
        p.trim_device_cache()
    finally:
        ctx.free()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

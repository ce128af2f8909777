"""One-rank RCCL MG Louvain calls beside the single-GPU call on the same R-MAT graph
(for a kernel trace of the MG level loop; measurement aid, not product).
usage: mg_louvain_once.py SCALE N"""
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
    scale, n = int(sys.argv[1]), int(sys.argv[2])
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(bench.free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    h = p.ResourceHandle()
    g, _, _ = bench.build_rmat_graph(p, h, scale, weighted=True, transposed=False)
    for i in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.louvain(h, g, 100, 1.0, False)
        torch.cuda.synchronize()
        print(f"SG call {i}: {time.perf_counter() - t0:.3f} s", flush=True)
    g = None
    h = None
    ctx = p.comms.init_rccl(1)
    try:
        hm = p.ResourceHandle(ctx.ptr)
        gm, _, _ = bench.build_rmat_graph(p, hm, scale, weighted=True, transposed=False, mg=(0, 1))
        for i in range(n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            p.louvain(hm, gm, 100, 1.0, False)
            torch.cuda.synchronize()
            print(f"MG call {i}: {time.perf_counter() - t0:.3f} s", flush=True)
        gm = None
        hm = None
        torch.cuda.synchronize()
        p.trim_device_cache()
    finally:
        ctx.free()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

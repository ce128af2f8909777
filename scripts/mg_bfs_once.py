"""One-rank RCCL MG BFS traversals (for a kernel trace; measurement aid, not product).
usage: mg_bfs_once.py SCALE N"""
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
    ctx = p.comms.init_rccl(1)
    try:
        hm = p.ResourceHandle(ctx.ptr)
        gm, roots, _ = bench.build_rmat_graph(p, hm, scale, transposed=False, mg=(0, 1), want_roots=1)
        src = torch.tensor([int(roots[0])], dtype=torch.int32, device="cuda")
        for i in range(n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = p.bfs(hm, gm, src.clone(), True, 0, True, False)
            torch.cuda.synchronize()
            print(f"traversal {i}: {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
            del res
        gm = None
        hm = None
        torch.cuda.synchronize()
        p.trim_device_cache()
    finally:
        ctx.free()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

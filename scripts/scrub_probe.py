"""Does device memory freed by another process cost this process at hipMalloc time,
and does touching it once up front move that cost? (measurement aid, not product)

usage: scrub_probe.py dirty GIB          allocate and fill GIB of device memory, exit
       scrub_probe.py louvain [prefault]  RMAT-26 Louvain leg (bench.louvain_leg), with the
                                          allocator's hipMalloc seconds; prefault first
                                          allocates, touches and frees most free memory
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    if sys.argv[1] == "dirty":
        n = int(sys.argv[2])
        bufs = [torch.ones(1 << 28, dtype=torch.float32, device="cuda") for _ in range(n)]  # 1 GiB each
        torch.cuda.synchronize()
        print(f"dirtied {len(bufs)} GiB", flush=True)
        return
    import argparse
    import bench
    import pylibcugraph as p
    if len(sys.argv) > 2 and sys.argv[2] == "prefault":
        t0 = time.perf_counter()
        free = torch.cuda.mem_get_info()[0]
        bufs = []
        while free > (8 << 30):
            bufs.append(torch.empty(1 << 31, dtype=torch.uint8, device="cuda"))  # 2 GiB
            free -= 1 << 31
        for b in bufs:
            b.zero_()
        torch.cuda.synchronize()
        n = len(bufs)
        del bufs
        torch.cuda.empty_cache()
        print(f"prefault {2 * n} GiB in {time.perf_counter() - t0:.2f} s", flush=True)
    args = argparse.Namespace(ctx=None, mg=None, world=1, louvain_scale=26)
    r = bench.louvain_leg(p, args, 26)
    print(f"louvain RMAT-26 {r['time_s']:.3f} s, allocator {r['allocator_during_call']}", flush=True)


if __name__ == "__main__":
    main()

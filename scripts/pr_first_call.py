"""The first PageRank call on a fresh graph (measurement aid, not product).

usage: python scripts/pr_first_call.py [SCALE] [REPS]
Builds the bench's R-MAT graph, warms the code objects on RMAT-10, then times the
first cugraph_pagerank on the fresh graph (out-weight sums, push schedule build,
calibration chunk, iterations) and a steady call, REPS times on fresh graphs; under
rocprofv3 --kernel-trace the markers between phases show where the time goes.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import pylibcugraph as p
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    h = p.ResourceHandle()
    small, _, _ = bench.build_rmat_graph(p, h, 10)
    p.pagerank(h, small, None, None, None, None, 0.85, 1e-6, 500, False)
    del small
    for _ in range(reps):
        g, _, _ = bench.build_rmat_graph(p, h, scale)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p.pagerank(h, g, None, None, None, None, 0.85, 1e-6, 500, False)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        it1 = h.last_iterations()
        p.pagerank(h, g, None, None, None, None, 0.85, 1e-6, 500, False)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"RMAT-{scale}: first call {1e3 * (t1 - t0):.2f} ms ({it1} iterations), steady "
              f"{1e3 * (t2 - t1):.2f} ms ({h.last_iterations()} iterations)", flush=True)
        g = None
        p.trim_device_cache()


if __name__ == "__main__":
    main()

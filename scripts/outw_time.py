"""Out-weight sums of a weighted bench graph (measurement aid, not product).

usage: python scripts/outw_time.py [SCALE] [WEIGHTS]   (WEIGHTS: ones | uniform)
Builds the bench's R-MAT graph with fp32 weights and computes its per-vertex
out-weight sums (what PageRank's first call does, compute_out_weight_sums) on three
fresh graphs, printing the wall time of each call; run under rocprofv3 --stats for
the kernels' own times.
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
    kind = sys.argv[2] if len(sys.argv) > 2 else "ones"
    h = p.ResourceHandle()
    for _ in range(3):
        g, _, _ = bench.build_rmat_graph(p, h, scale, weighted="ones" if kind == "ones" else True, transposed=True)
        g.adjacency(h, transposed=False)  # the CSR the sums run over, built off the clock
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x = g.out_weight_sums(h)
        torch.cuda.synchronize()
        print(f"RMAT-{scale} {kind}: out-weight sums {1e3 * (time.perf_counter() - t0):.3f} ms "
              f"(sum {float(x.double().sum()):.6g})", flush=True)
        del x, g
        p.trim_device_cache()


if __name__ == "__main__":
    main()

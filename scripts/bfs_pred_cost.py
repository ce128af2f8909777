"""What the predecessors cost a BFS traversal (measurement aid, not product).

usage: python scripts/bfs_pred_cost.py [SCALE] [REPS]
The bench graph and roots (bench.build_rmat_graph, as bfs_leg builds them); per root
the median wall time of REPS traversals with predecessors and without (the top-down
levels then skip their atomicMin per edge, the bottom-up levels their predecessor
store), and the difference.
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    h = p.ResourceHandle()
    g, roots, _ = bench.build_rmat_graph(p, h, scale, transposed=False, want_roots=8)

    def median_ms(r, pred):
        src = torch.tensor([int(r)], dtype=torch.int32, device="cuda")
        p.bfs(h, g, src.clone(), True, 0, pred, False)
        ts = []
        for _ in range(reps):
            res = None
            s_in = src.clone()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = p.bfs(h, g, s_in, True, 0, pred, False)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del res
        return sorted(ts)[len(ts) // 2] * 1e3

    tot_p = tot_n = 0.0
    for i, r in enumerate(roots):
        a, b = median_ms(r, True), median_ms(r, False)
        tot_p += a
        tot_n += b
        print(f"root {i} ({r}): with predecessors {a:.3f} ms, without {b:.3f} ms, difference {a - b:.3f}", flush=True)
    n = len(roots)
    print(f"mean: with {tot_p / n:.3f} ms, without {tot_n / n:.3f} ms", flush=True)


if __name__ == "__main__":
    main()

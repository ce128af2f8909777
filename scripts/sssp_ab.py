"""SSSP A/B (measurement aid, not product): ms per traversal (median of 3) on the
bench's weighted R-MAT graph from the first 4 bench roots, for each delta scale
(handle option sssp_delta: delta = scale * average weight / average degree).
With CGX_SSSP_TRACE=1 the library prints the rounds, edges relaxed and improvements.

usage: sssp_ab.py SCALE DELTA[:PULL] [DELTA[:PULL] ...]   (PULL: option sssp_pull, default 0)
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import pylibcugraph as p
    scale = int(sys.argv[1])
    h = p.ResourceHandle()
    g, roots, _ = bench.build_rmat_graph(p, h, scale, weighted=True, transposed=False, want_roots=8)
    roots = [int(x) for x in roots[:4]]
    for arg in sys.argv[2:]:
        d, pl = (arg.split(":") + ["0"])[:2]
        d, pl = float(d), int(pl)
        h.set_option("sssp_delta", d)
        h.set_option("sssp_pull", pl)
        per, rounds = [], []
        for r in roots:
            p.sssp(h, g, r, float("inf"), True, False)  # warm
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = p.sssp(h, g, r, float("inf"), True, False)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
                del res
            per.append(statistics.median(ts) * 1e3)
            rounds.append(h.last_iterations())
        print(f"delta scale {d:g} pull {pl}: mean {statistics.mean(per):.3f} ms/traversal, per root "
              f"{[round(x, 3) for x in per]}, rounds {rounds}", flush=True)


if __name__ == "__main__":
    main()

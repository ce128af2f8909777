"""PageRank A/B on one resident graph (measurement aid, not product).

usage: pr_ab.py SCALE [NAME=VAL,NAME=VAL ...] ...
Builds the bench's R-MAT graph for every argument (a comma list of handle
options, include/cugraph_amd/ext.h cugraph_amd_set_option, e.g. pr_enc=0,pr_hub=0,
or "base") runs 2 warm and 5 timed PageRank calls and prints ms per iteration from
the library's HIP events (h.last_hot_kernel_ms / launches).  Every call
runs exactly 16 iterations (epsilon 0, max 16: the "failed to converge" error is
expected and ignored), so ablations that change the ranks keep the same work.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def run(p, h, g):
    try:
        p.pagerank(h, g, None, None, None, None, 0.85, 0.0, 16, False)
    except RuntimeError as e:
        if "converge" not in str(e):
            raise


def main():
    import torch
    import bench
    import pylibcugraph as p
    scale = int(sys.argv[1])
    h = p.ResourceHandle()
    for arg in sys.argv[2:] or ["base"]:
        opts = {} if arg == "base" else {k: float(v) for k, v in (kv.split("=", 1) for kv in arg.split(","))}
        h.set_option(None, 0)
        for k, v in opts.items():
            h.set_option(k, v)
        try:
            # a fresh graph per setting: schedule-time settings (pr_win_bits, ...) apply
            g, _, _ = bench.build_rmat_graph(p, h, scale, transposed=True)
            E = g.number_of_edges()
            for _ in range(2):
                run(p, h, g)
            torch.cuda.synchronize()
            h.set_profiling(True)
            ms, n, it = 0.0, 0, 0
            for _ in range(5):
                run(p, h, g)
                ms += h.last_hot_kernel_ms()
                n += h.last_hot_kernel_launches()
                it += h.last_iterations()
            h.set_profiling(False)
            print(f"RMAT-{scale} {arg}: {ms / max(n, 1):.4f} ms/iteration ({it / 5:.0f} iterations, "
                  f"{E * it / 5 / (ms / 5 * 1e-3) / 1e9:.1f} Gedges/s)", flush=True)
        finally:
            g = None
            p.trim_device_cache()


if __name__ == "__main__":
    main()

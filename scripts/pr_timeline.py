"""Per-item timeline of the packed PageRank push (measurement aid, not product).

usage: pr_timeline.py SCALE [NAME=VAL,...]
Runs 16 iterations on the bench's R-MAT graph with CGX_PR_TIMELINE set (the push
records {launch, block, item, fetch time, end time} per item, s_memrealtime at
100 MHz) and prints, per launch: the span from the first fetch to the last end,
the blocks' busy share, the tail (span end - each block's last end), and the
longest items.  Items are summed by the block that took them; a block's time
between its items is its queue fetch.
"""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import bench
    import pylibcugraph as p
    scale = int(sys.argv[1])
    env = dict(kv.split("=", 1) for arg in sys.argv[2:] for kv in arg.split(","))
    os.environ.update(env)
    h = p.ResourceHandle()
    g, _, _ = bench.build_rmat_graph(p, h, scale, transposed=True)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "pr_timeline.csv")
    for rep in range(2):
        if rep == 1:
            os.environ["CGX_PR_TIMELINE"] = path
        try:
            p.pagerank(h, g, None, None, None, None, 0.85, 0.0, 16, False)
        except RuntimeError as e:
            if "converge" not in str(e):
                raise
    rows = list(csv.DictReader(open(path)))
    L = np.array([int(r["launch"]) for r in rows])
    B = np.array([int(r["block"]) for r in rows])
    I = np.array([int(r["item"]) for r in rows])
    S = np.array([int(r["start"]) for r in rows], dtype=np.int64)
    T = np.array([int(r["end"]) for r in rows], dtype=np.int64)
    tick_us = 0.01
    spans = []
    for l in sorted(set(L.tolist())):
        m = L == l
        s0, s1 = S[m].min(), T[m].max()
        span = (s1 - s0) * tick_us
        blocks = sorted(set(B[m].tolist()))
        last_end = np.array([T[m & (B == b)].max() for b in blocks])
        first = np.array([S[m & (B == b)].min() for b in blocks])
        busy = np.array([(T[m & (B == b)] - S[m & (B == b)]).sum() for b in blocks]) * tick_us
        tail = (s1 - last_end) * tick_us
        start_lag = (first - s0) * tick_us
        dur = (T[m] - S[m]) * tick_us
        spans.append(span)
        print(f"launch {l}: span {span:7.1f} us, items {m.sum()}, blocks {len(blocks)}, "
              f"busy/span {busy.mean() / span:.3f}, tail mean {tail.mean():6.1f} us max {tail.max():6.1f}, "
              f"start lag max {start_lag.max():5.1f} us, item us p50 {np.median(dur):6.1f} p90 "
              f"{np.percentile(dur, 90):6.1f} max {dur.max():6.1f}, items/block max {np.bincount(B[m]).max()}")
        if l == 8:
            order = np.argsort(-dur)[:8]
            print("   longest items (item, block, start us, dur us):",
                  [(int(I[m][k]), int(B[m][k]), round((S[m][k] - s0) * tick_us, 1), round(dur[k], 1)) for k in order])
            last = np.argsort(-(T[m]))[:8]
            print("   last-ending items (item, block, start us, end us):",
                  [(int(I[m][k]), int(B[m][k]), round((S[m][k] - s0) * tick_us, 1), round((T[m][k] - s0) * tick_us, 1))
                   for k in last])
    print(f"mean span {np.mean(spans[1:]):.1f} us")


if __name__ == "__main__":
    main()

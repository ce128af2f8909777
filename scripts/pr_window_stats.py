"""Per-window statistics of the PageRank push schedule (measurement aid, not product).

usage: pr_window_stats.py SCALE [WIN_BITS]
For the bench's R-MAT graph: the CSC edges grouped by 2^WIN_BITS-destination window and
sorted by source (the push's (window, source) order), then per window: edges, the
packed format's jump entries (16 - WIN_BITS delta bits: a source gap above
2^(16-WB) - 2 costs ceil(gap / (2^WB - 1)) jumps), the packed entries including the
pad to whole 512-entry segments, the distinct 128-B x~ lines (32 sources) the window
reads, and what a 32-bit entry per edge would cost.  Prints a summary by window
class (quantiles of edges per distinct line).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import pylibcugraph as p
    scale = int(sys.argv[1])
    wb = int(sys.argv[2]) if len(sys.argv) > 2 else (14 if scale >= 23 else 13 if scale >= 22 else 12)
    h = p.ResourceHandle()
    g, _, _ = bench.build_rmat_graph(p, h, scale, transposed=True)
    off, idx, _ = g.adjacency(h, transposed=True)
    g = None
    p.trim_device_cache()
    V = off.numel() - 1
    E = idx.numel()
    deg = (off[1:] - off[:-1]).to(torch.int64)
    dst = torch.repeat_interleave(torch.arange(V, device=off.device, dtype=torch.int64), deg)
    key = (dst >> wb) << 32 | idx.to(torch.int64)
    del dst, idx
    key = torch.sort(key).values
    nwin = int(key[-1] >> 32) + 1
    dmax = (1 << (16 - wb)) - 2
    pmax = (1 << wb) - 1
    dev = key.device
    e_w = torch.zeros(nwin, dtype=torch.int64, device=dev)
    j_w = torch.zeros(nwin, dtype=torch.int64, device=dev)
    l_w = torch.zeros(nwin, dtype=torch.int64, device=dev)
    chunk = 1 << 28
    for lo in range(0, E, chunk):  # chunked: the RMAT-26 arrays are 16.8 GB each
        hi = min(E, lo + chunk)
        k = key[max(lo - 1, 0):hi]
        win, src = k >> 32, k & 0xFFFFFFFF
        first = torch.ones(k.numel(), dtype=torch.bool, device=dev)
        first[1:] = win[1:] != win[:-1]
        gap = src.clone()
        gap[1:] = torch.where(first[1:], src[1:], src[1:] - src[:-1])
        jumps = torch.where(gap > dmax, (gap + pmax - 1) // pmax, torch.zeros_like(gap))
        line = src >> 5
        newline = first.clone()
        newline[1:] |= line[1:] != line[:-1]
        s0 = 1 if lo > 0 else 0  # the overlap element belongs to the previous chunk
        w = win[s0:]
        e_w += torch.bincount(w, minlength=nwin)
        j_w.index_add_(0, w, jumps[s0:])
        l_w.index_add_(0, w, newline[s0:].to(torch.int64))
        del k, win, src, first, gap, jumps, line, newline, w
    packed = e_w + j_w
    padded = (packed + 511) // 512 * 512
    print(f"RMAT-{scale}: V={V} E={E} windows={nwin} (2^{wb} rows), packed entries {int(packed.sum())} "
          f"({int(packed.sum()) / E:.3f}/edge), padded {int(padded.sum())} ({int(padded.sum()) / E:.3f}/edge), "
          f"jumps {int(j_w.sum())}, distinct x~ lines {int(l_w.sum())} ({int(l_w.sum()) * 128 / 1e9:.2f} GB/iteration "
          f"if every window's lines missed)")
    epl = e_w.double() / l_w.clamp(min=1).double()  # edges per distinct line
    order = torch.argsort(epl)
    cuts = [0, 0.05, 0.1, 0.25, 0.5, 0.75, 1.0]
    for a, b in zip(cuts[:-1], cuts[1:]):
        sel = order[int(a * nwin):int(b * nwin)]
        if sel.numel() == 0:
            continue
        ee, jj, ll, pp = (int(t[sel].sum()) for t in (e_w, j_w, l_w, padded))
        print(f"  windows {a:.2f}-{b:.2f} by edges/line ({float(epl[sel].min()):.2f}-{float(epl[sel].max()):.2f}): "
              f"edges {ee} ({ee / E:.1%}), jumps/edge {jj / max(ee, 1):.3f}, padded entries/edge {pp / max(ee, 1):.3f}, "
              f"lines/edge {ll / max(ee, 1):.3f}, 16-bit bytes/edge {2 * pp / max(ee, 1):.2f} vs 32-bit 4.00")
    # what a per-window choice would give: 32-bit entries where 2 * padded > 4 * edges
    wide = 2 * padded > 4 * e_w
    mixed = torch.where(wide, 4 * e_w, 2 * padded)
    print(f"  per-window choice: {int(wide.sum())} windows 32-bit ({int(e_w[wide].sum()) / E:.1%} of edges); "
          f"entry bytes {int(mixed.sum()) / 1e9:.3f} GB vs 16-bit {int(2 * padded.sum()) / 1e9:.3f} GB; lanes "
          f"{int(torch.where(wide, e_w, padded).sum()) / E:.3f}/edge vs {int(padded.sum()) / E:.3f}")


if __name__ == "__main__":
    main()

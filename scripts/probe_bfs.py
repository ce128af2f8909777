"""BFS kernel-sequence probe: RMAT graph, one root, warm + measured BFS.  Run under
`rocprofv3 --kernel-trace --output-format csv` and then with --summarize <csv>."""
import argparse
import csv
import re
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a):
    import torch
    import bench
    import pylibcugraph as p
    h = p.ResourceHandle(None)
    g, roots, _ = bench.build_rmat_graph(p, h, a.scale, transposed=False, want_roots=a.root_index + 1)
    r = roots[a.root_index]
    src = torch.tensor([int(r)], dtype=torch.int32, device="cuda")
    for _ in range(2):
        torch.cuda.synchronize()
        dist, pred, verts = p.bfs(h, g, src.clone(), True, 0, True, False)
        torch.cuda.synchronize()
    print("levels", h.last_bfs_levels(), file=sys.stderr)


def summarize(path, tail_from):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the measured BFS = kernels after the last k_bfs_init_sources
    idx = max(i for i, r in enumerate(rows) if "k_bfs_init" in r["Kernel_Name"])
    t0 = int(rows[idx]["Start_Timestamp"])
    for r in rows[idx:]:
        m = re.search(r"(k_\w+|__amd_\w+)(<[^(]*)?", r["Kernel_Name"])
        name = m.group(0) if m else r["Kernel_Name"][:60]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        st = (int(r["Start_Timestamp"]) - t0) / 1e3
        print(f"{st:9.1f} us  {d:8.1f} us  grid={r.get('Grid_Size_X', r.get('Grid_Size', '?')):>9}  {name}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=24)
    ap.add_argument("--root-index", type=int, default=1)
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize, 0)
    else:
        run(a)

"""Per-traversal BFS timeline from a rocprofv3 kernel trace (measurement aid).

usage: bfs_timeline.py TRACE_DIR [N_LAST]
Splits the trace at every k_bfs_setup launch (one per traversal) and prints, for the
last N_LAST traversals, every kernel's start offset, duration and the idle gap before
it, then the traversal's busy / idle split (idle = host round trips and launch gaps).
"""
import csv
import glob
import re
import sys


def short(n):
    n = n.replace('cgx::(anonymous namespace)::', '')
    return re.sub(r'<.*', '', n.split('(')[0].replace('void ', ''))[:32]


f = (glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True) + glob.glob(sys.argv[1] + "/**/*kernel_trace.csv.gz", recursive=True))[0]
import gzip
rows = sorted(csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)), key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Grid_Size_X"]) for r in rows]
starts = [i for i, k in enumerate(ks) if k[2].startswith("k_bfs_setup")]
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 3
tot_busy = tot_wall = 0.0
for j, a in enumerate(starts):
    b = starts[j + 1] if j + 1 < len(starts) else len(ks)
    seg = ks[a:b]
    # the traversal ends with k_finish_pred (later kernels belong to the caller)
    end = max(i for i, k in enumerate(seg) if k[2].startswith("k_finish_pred") or i == 0)
    seg = seg[:end + 1]
    t0 = seg[0][0]
    busy = sum(e - s for s, e, _, _ in seg) / 1e3
    wall = (seg[-1][1] - t0) / 1e3
    tot_busy += busy
    tot_wall += wall
    if j >= len(starts) - n_last:
        print(f"---- traversal {j}: wall {wall:.1f} us, kernels {busy:.1f} us, idle {wall - busy:.1f} us")
        prev = t0
        for s, e, n, g in seg:
            print(f"  +{(s - t0) / 1e3:8.1f} us  gap {(s - prev) / 1e3:6.1f}  {(e - s) / 1e3:7.1f} us  {n} grid={g}")
            prev = e
print(f"all {len(starts)} traversals: mean wall {tot_wall / max(len(starts), 1):.1f} us, "
      f"mean kernels {tot_busy / max(len(starts), 1):.1f} us")

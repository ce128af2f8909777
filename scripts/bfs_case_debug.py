"""One small BFS case with the level log and the distances against the oracle (debug aid).

usage: CGX_BFS_DEBUG=1 python scripts/bfs_case_debug.py DATASET [DO]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cugraph-forked_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    from gpu_util import host, make_graph, plc
    from oracle import bfs as obfs
    from oracle import graph as og
    name = sys.argv[1]
    do = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
    s, d, _ = og.read_csv(os.path.join(ROOT, "tests", "golden", name))
    h, G = make_graph(s, d, None, renumber=True, symmetric=True)
    src = [int(s[0])]
    dd, pp, vv = plc().bfs(h, G, np.asarray(src, np.int32), do, 0, True, False)
    v, dist = host(vv), host(dd)
    n_ext = int(max(s.max(), d.max())) + 1
    OG = og.create_graph(s, d, None, renumber=False, vertices=np.arange(n_ext))
    rd, _ = obfs.bfs(n_ext, OG.offsets, OG.indices, src, None)
    bad = np.nonzero(dist != rd[v])[0]
    print(f"{name} do={do}: V={v.size} levels {h.last_bfs_levels()} bottom-up {h.last_bfs_bottom_up_steps()}; "
          f"{bad.size} distances differ", flush=True)
    for i in bad[:20]:
        print(f"  internal {i} ext {v[i]}: got {dist[i]} want {rd[v[i]]}")
    print("dist histogram got", np.bincount(np.minimum(dist, 50)), "want", np.bincount(np.minimum(rd[v], 50)))


if __name__ == "__main__":
    main()

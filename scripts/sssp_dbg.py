import os, sys
sys.path.insert(0, '/root/repo/cugraph-forked_amd'); sys.path.insert(0, '/root/repo')
import numpy as np, torch
import pylibcugraph as p
from oracle import cpu_native
h = p.ResourceHandle()
scale = int(sys.argv[1])
n = 16 << scale
s, d = p.generators.generate_rmat_edgelist(h, scale, n, 0.57, 0.19, 0.19, 42, False, True)
w = p.generators.generate_edge_weights(h, n, 43)
s, d, w = p.generators.symmetrize_dedup(h, s, d, w, True)
G = p.SGGraph(h, p.GraphProperties(is_symmetric=True, is_multigraph=False), s, d, w, store_transposed=False, renumber=True)
off, idx, ww = G.adjacency(h, transposed=False)
off, idx, ww = off.cpu().numpy().astype(np.int64), idx.cpu().numpy(), ww.cpu().numpy()
V = off.size - 1
v, dist, pred = p.sssp(h, G, int(s[0]), 1e38, True, False)
nm = v.cpu().numpy()
bad = 0
for si in list(range(V - 40, V)) + [0, 1, 2]:
    v, dist, pred = p.sssp(h, G, int(nm[si]), 1e38, True, False)
    t, rd, rp, r = cpu_native.sssp(off, idx, ww, si)
    ok = np.array_equal(dist.cpu().numpy(), rd)
    deg = off[si + 1] - off[si]
    if not ok:
        bad += 1
        print('FAIL source', si, 'deg', deg, 'w', ww[off[si]:off[si+1]], 'reached gpu', int((dist.cpu().numpy() < 3e38).sum()), 'oracle', int((rd < 3e38).sum()), 'rounds', h.last_iterations(), flush=True)
print('bad', bad)

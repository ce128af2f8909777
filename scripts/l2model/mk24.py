import sys, numpy as np, time
sys.path.insert(0, "/root/repo")
from oracle import rmat, graph as og
sc = int(sys.argv[1])
s, d = rmat.rmat(sc, 16 << sc, seed=42)
s, d, _ = og.symmetrize_dedup(s, d, None)
V = 1 << sc
deg = np.bincount(s, minlength=V)
order = np.argsort(-deg, kind="stable")
order = order[deg[order] > 0]
nid = np.full(V, -1, np.int64); nid[order] = np.arange(order.size)
src, dst = nid[s].astype(np.int32), nid[d].astype(np.int32)
np.save(f"/tmp/ana/src{sc}.npy", src); np.save(f"/tmp/ana/dst{sc}.npy", dst)
print("saved", order.size, src.size)

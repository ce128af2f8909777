import numpy as np, sys
sc = int(sys.argv[1]); wb = int(sys.argv[2])
z = np.load(f"/tmp/ana/sorted_{sc}_contig_{wb}.npz"); ss, ws = z["ss"], z["ws"].astype(np.int64)
line = ss.astype(np.int64) >> 5
key = (ws << 24) | line
u = np.unique(key)
ul = u & ((1 << 24) - 1)
nv = int(ss.max()) + 1
deg = np.bincount(ss, minlength=nv)
edges = [0, 1 << 14, 1 << 16, 1 << 18, 1 << 20, 1 << 21, 1 << 22, 1 << 23, nv]
for a, b in zip(edges[:-1], edges[1:]):
    m = (ul >= (a >> 5)) & (ul < (b >> 5))
    e = deg[a:b].sum()
    print(f"src rank [{a:>8},{b:>8}) deg {deg[a]:>6}..{deg[b-1]:>3}: entries {e/ss.size:6.3f}  (win,line) pairs {m.sum()/u.size:6.3f} = {m.sum()/1e6:7.2f}M, lines/entry {m.sum()/max(e,1):.3f}")

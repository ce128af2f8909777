"""Source-range XCD partition of the push: window w's source-sorted entries are cut
at K global source boundaries (equal entry counts), piece k of every window goes to
XCD k's queue (tiles of <= 8 units, windows in order).  Each XCD then gathers x~ of
its own source range only.  usage: sched4.py SCALE WB [K] [balance: entries|lines]"""
import subprocess
import sys

import numpy as np

sc, wb = int(sys.argv[1]), int(sys.argv[2])
K = int(sys.argv[3]) if len(sys.argv) > 3 else 8
z = np.load(f"/tmp/ana/sorted_{sc}_contig_{wb}.npz")
ss, ws = z["ss"], z["ws"]
nv = int(ss.max()) + 1
E = ss.size
U = 8192
nwin = int(ws.max()) + 1
wstart = np.searchsorted(ws, np.arange(nwin + 1))
deg = np.bincount(ss, minlength=nv).astype(np.int64)
cum = np.cumsum(deg)
B = np.concatenate([[0], np.searchsorted(cum, np.arange(1, K) * E / K), [nv]])
print("source boundaries", B.tolist(), "x~ MB per range", [round((B[i + 1] - B[i]) * 4 / 2**20, 1) for i in range(K)])
items = []
for w in range(nwin):
    a, b = wstart[w], wstart[w + 1]
    cuts = a + np.searchsorted(ss[a:b], B)
    for k in range(K):
        for t0 in range(cuts[k], cuts[k + 1], 8 * U):
            items.append((t0, min(cuts[k + 1], t0 + 8 * U), k % 8))
items = np.array(items, np.int64)
# queue order: per XCD by window (items already in window order)
ss.astype(np.int32).tofile("/tmp/ana/s.bin")
items.tofile("/tmp/ana/t3.bin")
print(f"srcrange K={K} wb {wb} items {len(items)}", flush=True)
print(subprocess.run(["/tmp/ana/l2sim3", "/tmp/ana/s.bin", "/tmp/ana/t3.bin", str(nv), str(U), "32768", "-1", "1"],
                     capture_output=True, text=True).stdout)

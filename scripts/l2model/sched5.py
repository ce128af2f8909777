"""Head/tail XCD partition of the push: entries of the H highest-degree sources
(the head, cached by every XCD) go to XCD (window % 8) in tiles; entries of the tail
sources are cut at 8 tail boundaries (equal tail entries) and piece k goes to XCD k,
so each XCD gathers x~ of the head plus 1/8 of the tail.
usage: sched5.py SCALE WB H [tail cut: entries|vertices]
Head tiles go to the least-loaded XCD (after the tail pieces are placed)."""
import subprocess
import sys

import numpy as np

sc, wb, H = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
z = np.load(f"/tmp/ana/sorted_{sc}_contig_{wb}.npz")
ss, ws = z["ss"], z["ws"]
nv = int(ss.max()) + 1
E = ss.size
U = 8192
nwin = int(ws.max()) + 1
wstart = np.searchsorted(ws, np.arange(nwin + 1))
deg = np.bincount(ss, minlength=nv).astype(np.int64)
cum = np.cumsum(deg)
Eh = cum[H - 1] if H > 0 else 0
Et = E - Eh
cut = sys.argv[4] if len(sys.argv) > 4 else "entries"
if cut == "entries":
    B = np.concatenate([[H], np.searchsorted(cum, Eh + np.arange(1, 8) * Et / 8), [nv]])
else:
    B = np.linspace(H, nv, 9).astype(np.int64)
print(f"head {H} sources ({H * 4 / 2**20:.1f} MB, {Eh / E:.3f} of entries); tail cuts", B.tolist(),
      "MB", [round((B[i + 1] - B[i]) * 4 / 2**20, 1) for i in range(8)])
items, head = [], []
for w in range(nwin):
    a, b = wstart[w], wstart[w + 1]
    h1 = a + np.searchsorted(ss[a:b], H)
    for t0 in range(a, h1, 8 * U):
        head.append((t0, min(h1, t0 + 8 * U)))
    cuts = a + np.searchsorted(ss[a:b], B)
    for k in range(8):
        for t0 in range(cuts[k], cuts[k + 1], 8 * U):
            items.append((t0, min(cuts[k + 1], t0 + 8 * U), k))
load = np.zeros(8)
for a, b, k in items:
    load[k] += b - a
for a, b in head:
    k = int(np.argmin(load))
    load[k] += b - a
    items.append((a, b, k))
items = np.array(items, np.int64)
load = np.bincount(items[:, 2], weights=items[:, 1] - items[:, 0], minlength=8)
print("entries per XCD / ideal", np.round(load / (E / 8), 3).tolist())
ss.astype(np.int32).tofile("/tmp/ana/s.bin")
items.tofile("/tmp/ana/t3.bin")
print(f"headtail H={H} wb {wb} items {len(items)}", flush=True)
print(subprocess.run(["/tmp/ana/l2sim3", "/tmp/ana/s.bin", "/tmp/ana/t3.bin", str(nv), str(U), "32768", "-1", "1"],
                     capture_output=True, text=True).stdout)

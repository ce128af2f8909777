"""Production-like push schedule (16K windows, window items with shares, groups of 16
items dealt to the 8 XCD queues costliest-first by entries) vs a band-major variant
(items = (window, source band), all windows' band-0 items first), replayed through
l2sim4 with misses split by source band.
usage: sched6.py SCALE MODE [S1 ...]    MODE = window | band"""
import os
import subprocess
import sys

import numpy as np

sc, mode = int(sys.argv[1]), sys.argv[2]
cuts = [int(x) for x in sys.argv[3:]] or [65536, 1 << 20]
wb = 14
cache = f"/tmp/ana/sorted_{sc}_w{wb}.npy"
if os.path.exists(cache):
    ss = np.load(cache)
else:
    src = np.load(f"/tmp/ana/src{sc}.npy")
    dst = np.load(f"/tmp/ana/dst{sc}.npy")
    key = ((dst.astype(np.int64) >> wb) << 32) | src.astype(np.int64)
    key.sort()
    ss = (key & 0xffffffff).astype(np.int32)
    np.save(f"/tmp/ana/win_{sc}_w{wb}.npy", (key >> 32).astype(np.int32))
    np.save(cache, ss)
ws = np.load(f"/tmp/ana/win_{sc}_w{wb}.npy")
E = ss.size
nv = int(ss.max()) + 1
nwin = int(ws.max()) + 1
wstart = np.searchsorted(ws, np.arange(nwin + 1))
tg = max(8192, E // (256 * 4))


def shares(a, b):
    n = max(1, int(round((b - a) / tg)))
    c = np.linspace(a, b, n + 1).astype(np.int64)
    return [(c[i], c[i + 1]) for i in range(n) if c[i + 1] > c[i]]


def deal(items, G=16):
    items = np.array(items, np.int64)
    ng = -(-len(items) // G)
    gsz = np.array([(items[g * G:(g + 1) * G, 1] - items[g * G:(g + 1) * G, 0]).sum() for g in range(ng)])
    load = np.zeros(8)
    qs = [[] for _ in range(8)]
    for g in np.argsort(-gsz, kind="stable"):
        x = int(np.argmin(load))
        qs[x].append(g)
        load[x] += gsz[g]
    out = []
    for x in range(8):
        for g in qs[x]:
            for a, b in items[g * G:(g + 1) * G]:
                out.append((a, b, x))
    return out


if mode == "window":
    items = []
    for w in range(nwin):
        items += shares(wstart[w], wstart[w + 1])
    tiles = deal(items)
else:
    bounds = [0] + cuts + [nv]
    tiles = []
    for k in range(len(bounds) - 1):
        items = []
        for w in range(nwin):
            a, b = wstart[w], wstart[w + 1]
            lo = a + np.searchsorted(ss[a:b], bounds[k])
            hi = a + np.searchsorted(ss[a:b], bounds[k + 1])
            if hi > lo:
                items += shares(lo, hi)
        tiles += deal(items)  # band k's items are all queued before band k + 1's
    # queue order must be band-major per XCD: deal() kept each band's items together
tiles = np.array(tiles, np.int64)
# per XCD queue in list order: stable sort by xcd keeps the band-major order inside each queue
tiles = tiles[np.argsort(tiles[:, 2], kind="stable")]
ss.astype(np.int32).tofile("/tmp/ana/s6.bin")
tiles.tofile("/tmp/ana/t6.bin")
print(f"RMAT-{sc} {mode} cuts {cuts}: {len(tiles)} items, E={E}", flush=True)
r = subprocess.run(["/tmp/ana/l2sim4", "/tmp/ana/s6.bin", "/tmp/ana/t6.bin", str(nv), "8192", "32768", "256"] +
                   [str(x) for x in [8064, 65536, 262144, 1 << 20, 1 << 22]], capture_output=True, text=True)
print(r.stdout, r.stderr)

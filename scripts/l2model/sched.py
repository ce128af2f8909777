import sys, numpy as np, subprocess
sc = int(sys.argv[1]); mode = sys.argv[2]; tile_units = int(sys.argv[3]) if len(sys.argv) > 3 else 8
wb = int(sys.argv[4]) if len(sys.argv) > 4 else 12
src = np.load(f"/tmp/ana/src{sc}.npy"); dst = np.load(f"/tmp/ana/dst{sc}.npy")
nv = int(max(src.max(), dst.max())) + 1
U = 8192
if mode.startswith("contig"):
    win = dst.astype(np.int64) >> wb
elif mode == "strided":
    runs = (nv + 63) >> 6; need = -(-runs // (1 << (wb - 6))); nwin = min(-(-need // 512) * 512, runs)
    win = (dst.astype(np.int64) >> 6) % nwin
import os
cache = f"/tmp/ana/sorted_{sc}_{mode[:6]}_{wb}.npz"
if os.path.exists(cache):
    z = np.load(cache); ss, ws = z["ss"], z["ws"]
else:
    key = (win << 32) | src.astype(np.int64)
    o = np.argsort(key, kind="stable")
    ss = src[o]; ws = win[o].astype(np.int32)
    np.savez(cache, ss=ss, ws=ws)
nwin = int(ws.max()) + 1
wstart = np.searchsorted(ws, np.arange(nwin + 1))
tiles = []
for w in range(nwin):
    a, b = wstart[w], wstart[w + 1]
    step = U * tile_units
    for t0 in range(a, b, step):
        tiles.append((t0, min(b, t0 + step), w, ss[t0]))
tiles = np.array(tiles, dtype=np.int64)
if mode == "contig_srcmajor":  # queue: by (window band of 512 tiles?) -> by first source inside bands
    band = np.arange(len(tiles)) // int(sys.argv[5])
    tiles = tiles[np.lexsort((tiles[:, 3], band))]
xcd = np.full(len(tiles), -1, np.int64)
if mode == "contig_lockstep":  # groups of G consecutive windows per XCD (round robin by group), chunked sources
    G = int(sys.argv[5]); CH = int(sys.argv[6])  # CH: source chunk (sources)
    out = []
    grp = 0
    for g0 in range(0, nwin, G):
        x = grp % 8; grp += 1
        ws_ = range(g0, min(nwin, g0 + G))
        # per window, entries split by source chunk
        bounds = {w: np.searchsorted(ss[wstart[w]:wstart[w+1]], np.arange(0, nv + CH, CH)) + wstart[w] for w in ws_}
        nch = (nv + CH - 1) // CH
        for c in range(nch):
            for w in ws_:
                a, b = bounds[w][c], bounds[w][c + 1]
                if b > a: out.append((a, b, x))
    tiles = np.array(out, dtype=np.int64); xcd = tiles[:, 2]
ss.astype(np.int32).tofile("/tmp/ana/s.bin"); np.stack([tiles[:, 0], tiles[:, 1], xcd], 1).astype(np.int64).tofile("/tmp/ana/t.bin")
print(mode, "nwin", nwin, "tiles", len(tiles), flush=True)
print(subprocess.run(["/tmp/ana/l2sim", "/tmp/ana/s.bin", "/tmp/ana/t.bin", str(nv), str(U), "32768"], capture_output=True, text=True).stdout)

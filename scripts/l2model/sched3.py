import sys, numpy as np, subprocess
sc = int(sys.argv[1]); wb = int(sys.argv[2]); tfac = float(sys.argv[3]); gate = sys.argv[4]; R = sys.argv[5]; mode = sys.argv[6]
z = np.load(f"/tmp/ana/sorted_{sc}_contig_{wb}.npz"); ss, ws = z["ss"], z["ws"]
nv = int(ss.max()) + 1; E = ss.size; U = 8192
nwin = int(ws.max()) + 1
wstart = np.searchsorted(ws, np.arange(nwin + 1))
if mode == "tiles":   # current: tiles of <= 8 units, one global queue (xcd -1)
    items = []
    for w in range(nwin):
        for a in range(wstart[w], wstart[w+1], 8 * U): items.append((a, min(wstart[w+1], a + 8 * U), -1))
    items = np.array(items)
else:                  # items of ~tfac * E/2048 entries; groups of 64 consecutive items -> XCDs by LPT
    Tg = tfac * E / 512 / 4
    it = []
    if mode == "xcdtiles":
        for w in range(nwin):
            for a in range(wstart[w], wstart[w+1], 8 * U): it.append((a, min(wstart[w+1], a + 8 * U)))
    for w in (range(nwin) if mode in ("xcd", "win") else []):
        a, b = wstart[w], wstart[w + 1]
        n = max(1, int(round((b - a) / Tg)))
        cuts = np.linspace(a, b, n + 1).astype(np.int64)
        for i in range(n):
            if cuts[i + 1] > cuts[i]: it.append((cuts[i], cuts[i + 1]))
    it = np.array(it); G = int(sys.argv[7]) if len(sys.argv) > 7 else 64
    ng = -(-len(it) // G)
    gsz = np.array([(it[g*G:(g+1)*G, 1] - it[g*G:(g+1)*G, 0]).sum() for g in range(ng)])
    load = np.zeros(8); gx = np.zeros(ng, int)
    if len(sys.argv) > 8 and sys.argv[8] == "rr":
        gx = np.arange(ng) % 8
    elif G > 100000:  # contiguous: 8 ranges of equal entries
        cum = np.cumsum(gsz); gx = np.minimum(7, (8 * (cum - gsz / 2) / cum[-1]).astype(int))
    else:
        for g in np.argsort(-gsz, kind="stable"):
            x = int(np.argmin(load)); gx[g] = x; load[x] += gsz[g]
    items = np.array([(a, b, -1 if mode == "win" else gx[i // G]) for i, (a, b) in enumerate(it)], np.int64)
ss.astype(np.int32).tofile("/tmp/ana/s.bin"); items.astype(np.int64).tofile("/tmp/ana/t3.bin")
print(f"{mode} wb {wb} items {len(items)} gate {gate}", flush=True)
print(subprocess.run(["/tmp/ana/l2sim3", "/tmp/ana/s.bin", "/tmp/ana/t3.bin", str(nv), str(U), "32768", gate, R], capture_output=True, text=True).stdout)

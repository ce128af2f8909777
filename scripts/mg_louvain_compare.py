"""Per-call kernel totals of SG and one-rank MG Louvain from the trace of
scripts/gpu_mg_louvain_trace.sh (graph builds excluded: each segment starts at its
first k_vertex_weights).  usage: mg_louvain_compare.py TRACE.csv.gz [TOP]"""
import collections
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from round_extracts import load  # noqa: E402

rows = load(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 22
a, b = [i for i, r in enumerate(rows) if r["_n"] == "k_rmat" and r["_d"] > 500_000][:2]


def first(lo, hi):
    return next(i for i in range(lo, hi) if rows[i]["_n"] == "k_vertex_weights")


def agg(seg, calls=2):
    c, n = collections.defaultdict(float), collections.Counter()
    for r in seg:
        c[r["_n"]] += r["_d"] / 1e6 / calls
        n[r["_n"]] += 1
    return c, n


sg, sgn = agg(rows[first(a, b):b])
mg, mgn = agg(rows[first(b, len(rows)):])
print(f"{'kernel (per call)':40s} {'SG ms':>8s} {'n':>5s} {'MG ms':>8s} {'n':>5s}")
for k in sorted(set(sg) | set(mg), key=lambda k: -(mg.get(k, 0) - sg.get(k, 0)))[:top]:
    print(f"{k[:40]:40s} {sg.get(k, 0):8.2f} {sgn.get(k, 0) // 2:5d} {mg.get(k, 0):8.2f} {mgn.get(k, 0) // 2:5d}")
print(f"kernel time per call: SG {sum(sg.values()):.1f} ms, MG {sum(mg.values()):.1f} ms")

"""Per-dispatch PMC counters of the BFS child's large kernels (scripts/gpu_bfs_pmc.sh
output): one line per k_topdown / k_bu_probe / k_bu_residual dispatch over 60 us.
usage: bfs_pmc_summary.py DIR"""
import collections
import csv
import gzip
import sys

d = sys.argv[1]
data = collections.defaultdict(dict)
meta = {}
for p in (1, 2, 3):
    for r in csv.DictReader(gzip.open(f"{d}/pass{p}.csv.gz", "rt")):
        n = r["Kernel_Name"].replace("void ", "").replace("cgx::(anonymous namespace)::", "").split("(")[0].split("<")[0]
        if n not in ("k_topdown", "k_bu_probe", "k_bu_residual"):
            continue
        key = (p, int(r["Dispatch_Id"]))
        data[key][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[key] = (n, int(r["Grid_Size"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
# the passes run the same dispatch sequence: align by order within each pass
seq = {p: sorted(k for k in data if k[0] == p) for p in (1, 2, 3)}
n = min(len(v) for v in seq.values())
print("kernel grid | us | FETCH MB (x2 gfx950) | WRITE MB | L2 hit % | wave-cycles: wait % issue-stall % active % | VMEM insts M")
for i in range(n):
    k1, k2, k3 = seq[1][i], seq[2][i], seq[3][i]
    name, grid, us = meta[k1]
    if us < 60:
        continue
    a, b, c = data[k1], data[k2], data[k3]
    fetch = 2 * a.get("FETCH_SIZE", 0) / 1e3
    write = b.get("WRITE_SIZE", 0) / 1e3
    hit = a.get("TCC_HIT_sum", 0)
    miss = b.get("TCC_MISS_sum", 0)
    wc = c.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"{name} {grid} | {us:.0f} | {fetch:.0f} | {write:.0f} | {100 * hit / max(hit + miss, 1):.1f} | "
          f"{100 * c.get('SQ_WAIT_ANY', 0) / wc:.0f} {100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:.0f} "
          f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.0f} | {c.get('SQ_INSTS_VMEM', 0) / 1e6:.1f}")

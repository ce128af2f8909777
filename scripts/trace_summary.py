"""Kernel-trace summary (measurement aid): per-kernel totals and host gaps of a
rocprofv3 --kernel-trace CSV (optionally gzipped), from the N-th launch of a marker
kernel on.  usage: trace_summary.py TRACE [MARKER] [N] [TOP]"""
import collections
import csv
import gzip
import re
import sys


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    if "rocprim" in n:
        m = re.search(r"(radix_sort_onesweep|radix_sort_histogram|partition|reduce_by_key|segmented_reduce|scan|"
                      r"reduce|transform|sort)", n)
        return "rocprim:" + (m.group(1) if m else n[:40])
    return n.split("(")[0].split("<")[0].replace("cgx::", "")


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else None
    nth = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 25
    f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    if marker:
        idx = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == marker]
        rows = rows[idx[nth]:]
    t0, t1 = int(rows[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in rows)
    agg = collections.defaultdict(lambda: [0, 0.0])
    gaps = collections.defaultdict(float)
    prev = None
    for r in rows:
        n = short(r["Kernel_Name"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        agg[n][0] += 1
        agg[n][1] += (e - s) / 1e6
        if prev is not None and s > prev:
            gaps[n] += (s - prev) / 1e6
        prev = max(prev or 0, e)
    busy = sum(v[1] for v in agg.values())
    print(f"span {(t1 - t0) / 1e6:.2f} ms, kernels {busy:.2f} ms, gaps {sum(gaps.values()):.2f} ms")
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"  {v[1]:8.3f} ms {v[0]:5d}  {k}")
    print("largest gaps (before kernel):")
    for k, v in sorted(gaps.items(), key=lambda x: -x[1])[:10]:
        print(f"  {v:8.3f} ms  {k}")


if __name__ == "__main__":
    main()

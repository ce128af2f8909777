#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output directory into a markdown table.

Per kernel (demangled name shortened): launches, average / total duration from the
rocprofv3 kernel trace, and the average of every PMC counter collected in the
separate --pmc passes.  HBM bytes per launch = 2 x FETCH_SIZE (gfx950 reports half
of wide streaming reads, MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KB.

usage: python scripts/prof_summary.py gpurun_out/prof_<tag> > profiles/<name>.md
"""
from __future__ import annotations

import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    m = re.match(r"([\w:]+)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:80]


def main(d: str) -> None:
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "kt", "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    pmc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    counters = sorted({c for k in pmc.values() for c in k})
    print(f"# rocprofv3 summary: {os.path.basename(os.path.normpath(d))}\n")
    print("Durations from `rocprofv3 --kernel-trace --stats`; counters from separate `--pmc` passes "
          "(averages per launch).  HBM KB = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction).\n")
    hdr = ["kernel", "launches", "avg ms", "total ms"] + counters
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        hdr.append("HBM KB/launch")
    if "TCC_HIT_sum" in counters and "TCC_MISS_sum" in counters:
        hdr.append("L2 hit")
    print("| " + " | ".join(hdr) + " |")
    print("|" + "---|" * len(hdr))
    rows = sorted(dur.items(), key=lambda kv: -sum(kv[1]))
    for k, v in rows:
        c = pmc.get(k, {})
        avg = {n: (sum(c[n]) / len(c[n]) if c.get(n) else None) for n in counters}
        cells = [k, str(len(v)), f"{sum(v) / len(v):.4f}", f"{sum(v):.3f}"]
        cells += [f"{avg[n]:.4g}" if avg[n] is not None else "" for n in counters]
        if "HBM KB/launch" in hdr:
            f_, w_ = avg.get("FETCH_SIZE"), avg.get("WRITE_SIZE")
            cells.append(f"{2 * f_ + w_:.4g}" if f_ is not None and w_ is not None else "")
        if "L2 hit" in hdr:
            h_, m_ = avg.get("TCC_HIT_sum"), avg.get("TCC_MISS_sum")
            cells.append(f"{h_ / (h_ + m_):.3f}" if h_ is not None and m_ is not None and h_ + m_ > 0 else "")
        print("| " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main(sys.argv[1])

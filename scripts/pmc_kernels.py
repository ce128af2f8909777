"""Per-kernel average of each counter in a rocprofv3 counter_collection.csv
(measurement aid).  usage: pmc_kernels.py CSV KERNEL_SUBSTRING ..."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for k in sys.argv[2:]:
    agg = collections.defaultdict(list)
    for r in rows:
        if k in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    if agg:
        print(k, {c: f"{sum(v) / len(v):.4g}" for c, v in sorted(agg.items())}, "launches",
              max(len(v) for v in agg.values()))

"""Summarise rocprofv3 counter_collection.csv files: per kernel (name prefix match),
the average of every counter over launches whose first counter is non-trivial."""
import csv, sys, collections
kern = sys.argv[1]
acc = collections.defaultdict(list)
for f in sys.argv[2:]:
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    live = [x for x in v if x > 0.01 * max(v)] if max(v) > 0 else v
    print(f"{k:32s} launches {len(v):4d} avg(live) {sum(live)/max(len(live),1):.6g}")

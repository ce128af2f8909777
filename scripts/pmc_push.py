"""Average per-launch PMC values of the PageRank push from rocprofv3 counter CSVs
(launches below 10 % of the largest value of the first counter are post-convergence
no-ops and are dropped).  usage: pmc_push.py DIR [DIR...]"""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    rows = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for r in rows:
        k = r["Kernel_Name"]
        if "k_pr_push" not in k and "k_pr_apply" not in k:
            continue
        name = "push" if "k_pr_push" in k else "apply"
        per[(name, r.get("Dispatch_Id", r.get("Correlation_Id", "")))][r["Counter_Name"]] += float(r["Counter_Value"])
        per[(name, r.get("Dispatch_Id", r.get("Correlation_Id", "")))]["~ns"] = (
            float(r.get("End_Timestamp", 0) or 0) - float(r.get("Start_Timestamp", 0) or 0))
    for name in ("push", "apply"):
        launches = [v for (n, _), v in per.items() if n == name]
        if not launches:
            continue
        ctrs = sorted(launches[0].keys())
        top = max(x[ctrs[0]] for x in launches)
        live = [x for x in launches if x[ctrs[0]] > 0.1 * top]
        print(f"{d} {name}: {len(live)} of {len(launches)} launches")
        for c in ctrs:
            print(f"  {c:28s} {sum(x[c] for x in live) / len(live):16.4g}")

"""Per-kernel time of the last SSSP traversal in a rocprofv3 kernel trace
(measurement aid): usage sssp_trace_summary.py TRACE.csv"""
import csv
import re
import sys
from collections import defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
inits = [i for i, (s, e, n) in enumerate(ks) if 'k_sssp_init' in n]
last = ks[inits[-1]:]
end = [i for i, (s, e, n) in enumerate(last) if 'k_sssp_pred' in n][0]
last = last[:end + 2]
agg, cnt = defaultdict(float), defaultdict(int)
for s, e, n in last:
    m = re.search(r'(k_\w+|__amd\w+)', n)
    k = m.group(1) if m else n[:30]
    agg[k] += (e - s) / 1e6
    cnt[k] += 1
span = (last[-1][1] - last[0][0]) / 1e6
gaps = sum(max(0, last[i + 1][0] - last[i][1]) for i in range(len(last) - 1)) / 1e6
print(f"last traversal: span {span:.3f} ms, kernels {sum(agg.values()):.3f} ms, gaps {gaps:.3f} ms")
for k, v in sorted(agg.items(), key=lambda x: -x[1]):
    print(f"  {k:28s} {cnt[k]:5d} launches {v:8.3f} ms")

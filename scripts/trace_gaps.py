"""Summarise a rocprofv3 kernel trace: longest kernels and longest idle gaps."""
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:110]) for r in rows))
print("kernels", len(ks), "span ms", (ks[-1][1] - ks[0][0]) / 1e6)
for s, e, n in sorted(ks, key=lambda k: k[0] - k[1])[:12]:
    print(f"  kernel {(e - s) / 1e6:9.2f} ms  {n}")
gaps = [(ks[i + 1][0] - ks[i][1], ks[i][2], ks[i + 1][2]) for i in range(len(ks) - 1)]
for g, a, b in sorted(gaps, reverse=True)[:12]:
    print(f"  gap {g / 1e6:9.2f} ms after {a[:60]} before {b[:60]}")

set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_pr -o pr -- python3 bench.py --steps 2 --warmup 1 --no-louvain --no-bfs --no-traffic --no-cpu-baseline > gpurun_out/tr_pr.log 2>&1; rc=$?
python3 - <<'PY'
import csv, glob
f = glob.glob("/tmp/tr_pr/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
idx = [i for i, k in enumerate(ks) if "k_pr_init" in k[2]]
a, b = idx[-2], idx[-1]
t0 = ks[a][0]
prev = t0
for s, e, n in ks[a - 6:b]:
    nm = n.replace("void ", "").replace("cgx::(anonymous namespace)::", "").split("(")[0][:40]
    print(f"{(s - t0) / 1e3:9.1f} us  gap {(s - prev) / 1e3:7.1f}  dur {(e - s) / 1e3:8.1f} us  {nm}")
    prev = e
PY
exit $rc

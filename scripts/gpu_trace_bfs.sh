set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_bfs -o bfs -- python3 bench.py --steps 1 --warmup 0 --no-louvain --no-traffic --no-cpu-baseline --bfs-roots 1 > gpurun_out/tr_bfs.log 2>&1; rc=$?
python3 - <<'PY'
import csv, glob
f = glob.glob("/tmp/tr_bfs/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
# last BFS traversal: from the last k_bfs_init_sources on
idx = [i for i, k in enumerate(ks) if "k_bfs_init_sources" in k[2]][-1]
t0 = ks[idx][0]
for s, e, n in ks[idx:]:
    nm = n.replace("void ", "").replace("cgx::(anonymous namespace)::", "").split("(")[0][:40]
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  {nm}")
PY
exit $rc

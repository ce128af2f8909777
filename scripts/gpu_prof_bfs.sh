set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bfs -o bfs -- python3 bench.py --steps 1 --warmup 0 --no-louvain --no-traffic --no-cpu-baseline --bfs-roots 2 > gpurun_out/prof_bfs.log 2>&1; rc=$?
f=$(find /tmp/prof_bfs -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/bfs_kernel_stats.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/bfs_kernel_stats.csv')))
for r in rows:
    n=r['Name']
    if any(k in n for k in ('k_bu_','k_bottomup','k_topdown','k_mark','k_bitmap','fill','copyBuffer','k_finish_pred','k_bfs','k_frontier')):
        print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}us max {float(r['MaxNs'])/1e3:9.1f}us  {n[:80]}")
PY
exit $rc

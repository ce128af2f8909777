# kernel stats of the BFS traffic child (one traversal per root) with and without CGX_BFS_PROBE_VEC
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-probetr}; mkdir -p $OUT
for m in base vec base vec; do
  rm -rf /tmp/tr_$m
  if [ $m = vec ]; then export CGX_BFS_PROBE_VEC=1; else unset CGX_BFS_PROBE_VEC; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tr_$m -o tr -- python3 bench.py --traffic-child bfs --bfs-scale 24 --bfs-roots 8 > $OUT/trace_$m.log 2>&1 || exit $?
  f=$(find /tmp/tr_$m -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/stats_$m.csv
  echo "== $m"; grep -E "k_bu_probe|k_bu_residual|k_topdown" $OUT/stats_$m.csv | cut -d, -f1-5 | cut -c1-40,100-
done

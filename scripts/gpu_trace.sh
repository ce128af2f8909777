# rocprofv3 kernel trace of one bench child (graph build + one call per root)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-trace}; mkdir -p $OUT
rm -rf /tmp/tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tr -o tr -- python3 bench.py ${CHILD:---traffic-child bfs --bfs-scale 24 --bfs-roots 8} > $OUT/trace.log 2>&1
rc=$?
for f in $(find /tmp/tr -name "*kernel_trace.csv" -o -name "*kernel_stats.csv"); do cp $f $OUT/; done
exit $rc

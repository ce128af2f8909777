set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_lv -o lv -- python3 bench.py --steps 1 --warmup 0 --no-bfs --no-traffic --no-cpu-baseline --louvain-scale ${LS:-23} > gpurun_out/prof_lv.log 2>&1; rc=$?
grep "\[bench\]" gpurun_out/prof_lv.log; f=$(find /tmp/prof_lv -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/lv_kernel_stats.csv; head -25 "$f" | cut -d, -f1-5 | cut -c1-200; exit $rc

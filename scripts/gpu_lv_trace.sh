set -o pipefail
CGX_LOUVAIN_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-bfs --no-traffic --no-cpu-baseline --louvain-scale 23 > gpurun_out/lvtrace.log 2>&1; rc=$?; grep "\[bench\] louvain" gpurun_out/lvtrace.log; exit $rc

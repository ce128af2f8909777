set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CGX_LOUVAIN_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-bfs --no-traffic --no-cpu-baseline --louvain-scale 23 > gpurun_out/lvtrace.log 2>&1; rc=$?; grep "\[bench\]" gpurun_out/lvtrace.log; grep "louvain\]" gpurun_out/lvtrace.log | sort -t' ' -k1,1 | awk '{print}' | grep -v "nv=882\|nv=123\|nv=28 " | tail -12; exit $rc

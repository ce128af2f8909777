set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_louvain.py tests/test_gpu_mg.py -k "louvain" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_lv.log 2>&1; rc=$?; tail -2 gpurun_out/pt_lv.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-bfs --no-traffic --no-cpu-baseline 2>&1 | grep "\[bench\] louvain" || exit 1; done

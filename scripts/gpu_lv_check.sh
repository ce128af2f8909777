set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_louvain.py tests/test_gpu_mg.py tests/test_gpu_cugraph_api.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_lv.log 2>&1; rc=$?; tail -2 gpurun_out/pt_lv.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-bfs --no-traffic --no-cpu-baseline 2>&1 | grep "\[bench\] louvain" || exit 1
done

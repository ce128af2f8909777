set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_bfs.py tests/test_gpu_cugraph_api.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_bfs.log 2>&1; rc=$?; tail -2 gpurun_out/pt_bfs.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-louvain --no-traffic --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["bfs"]; print("probe", round(d["mteps_harmonic_mean"]), round(d["ms_mean"],3))' || exit 1
  CGX_BFS_ONE_PASS_BU=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-louvain --no-traffic --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["bfs"]; print("onepass", round(d["mteps_harmonic_mean"]), round(d["ms_mean"],3))' || exit 1
done
CGX_BFS_DEBUG=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-louvain --no-traffic --no-cpu-baseline --bfs-roots 1 2>&1 | grep "\[bfs\]" | tail -7

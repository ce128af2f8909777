set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_bfs.py tests/test_gpu_cugraph_api.py tests/test_gpu_centrality.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_bfs.log 2>&1; rc=$?; tail -1 gpurun_out/pt_bfs.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-louvain --no-traffic > gpurun_out/bfs_ab.json 2>/dev/null || exit 1
  tail -1 gpurun_out/bfs_ab.json | python -c "import json,sys; d=json.loads(sys.stdin.read())['bfs']; print('nomemset', round(d['mteps_harmonic_mean']), round(d['ms_mean'],4))"
done

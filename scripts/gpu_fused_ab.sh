set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_pr.log 2>&1; rc=$?; tail -3 gpurun_out/pt_pr.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-bfs --no-louvain --no-traffic"
for rep in 1 2; do
  timeout -k 10 120 $B 2>&1 | grep "\[bench\] pagerank" | sed "s/^/fused /" || exit 1
  CGX_PR_FUSED=0 timeout -k 10 120 $B 2>&1 | grep "\[bench\] pagerank" | sed "s/^/split /" || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_mg.log 2>&1; rc=$?; tail -3 gpurun_out/pt_mg.log; exit $rc

set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_pr.log 2>&1; rc=$?; tail -2 gpurun_out/pt_pr.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-bfs --no-louvain --no-traffic"
for rep in 1 2 3; do
  timeout -k 10 120 $B 2>&1 | grep "\[bench\] pagerank" | sed "s/^/batch4 /" || exit 1
  CUGRAPH_AMD_LIB=scripts/variants/ab1.so timeout -k 10 120 $B 2>&1 | grep "\[bench\] pagerank" | sed "s/^/batch1 /" || exit 1
done

set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "encoded or repeat or multi_window" > gpurun_out/pt_pr.log 2>&1; rc=$?; tail -2 gpurun_out/pt_pr.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for mode in enc plain; do
    CGX_PR_PUSH=$mode timeout -k 10 120 python bench.py --steps 10 --warmup 2 --epsilon 1e9 --no-cpu-baseline --no-bfs --no-louvain --no-traffic 2>&1 | grep "\[bench\] pagerank" | sed "s/^/$mode /" || exit 1
  done
done

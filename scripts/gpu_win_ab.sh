set -o pipefail
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-bfs --no-louvain --no-traffic"
for rep in 1 2; do
  timeout -k 10 120 $B 2>&1 | grep "\[bench\] pagerank" | sed "s/^/base /" || exit 1
  for v in t4 pt4 pt16; do
    CUGRAPH_AMD_LIB=scripts/variants/$v.so timeout -k 10 120 $B 2>&1 | grep "\[bench\] pagerank" | sed "s/^/$v /" || exit 1
  done
done
CUGRAPH_AMD_LIB=scripts/variants/pt16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_pr.log 2>&1; rc=$?; tail -2 gpurun_out/pt_pr.log; exit $rc

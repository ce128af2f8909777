set -o pipefail
for rep in 1 2; do
  for L in s1k8 s1k32 s1k64; do
    CUGRAPH_AMD_LIB=scripts/variants/$L.so timeout -k 10 120 python bench.py --steps 10 --warmup 2 --epsilon 1e9 --no-cpu-baseline --no-bfs --no-louvain --no-traffic 2>&1 | grep "\[bench\] pagerank" | sed "s/^/$L /" || exit 1
  done
  CUGRAPH_AMD_LIB=scripts/variants/s1k32.so CGX_PR_PUSH=static timeout -k 10 120 python bench.py --steps 10 --warmup 2 --epsilon 1e9 --no-cpu-baseline --no-bfs --no-louvain --no-traffic 2>&1 | grep "\[bench\] pagerank" | sed "s/^/static1 /" || exit 1
done

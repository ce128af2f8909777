#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
for m in ${MODES:-0 1 2 3 4 8 12}; do
  CGX_PR_ABLATE=$m timeout -k 10 120 python bench.py --steps 10 --warmup 2 --epsilon 1e9 --no-cpu-baseline --no-bfs ${EXTRA:-} 2>&1 | grep "\[bench\] pagerank" | sed "s/^/ablate=$m /"
done

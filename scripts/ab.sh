#!/bin/bash
# Same-box A/B of library variants: LIBS="path1 path2 ..." (default: the in-tree build)
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for L in ${LIBS:-cugraph-forked_amd/lib/libcugraph_c.so}; do
    CUGRAPH_AMD_LIB=$L timeout -k 10 120 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-bfs ${EXTRA:-} 2>&1 \
      | grep "\[bench\] pagerank" | sed "s|^|$(basename $L) |" || exit 1
  done
done

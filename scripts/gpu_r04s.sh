#!/bin/bash
# round-4: three bottom-up levels per round trip -- BFS tests (twice), MG BFS, bench, level log
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04s}; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py "tests/test_gpu_bench_parity.py::test_bfs_rmat24_all_bench_roots" -m gpu -x -q --timeout 200 --timeout-method thread \
    > $OUT/pytest_bfs_$i.log 2>&1; rc=$?; tail -1 $OUT/pytest_bfs_$i.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_bfs_$i.log | head; exit $rc; }
done
TAG=${TAG:-r04s}/bfs MODES="- CGX_BFS_BU_SPEC=1 - CGX_BFS_BU_SPEC=1" bash scripts/gpu_bfs_ab.sh || exit $?
CGX_BFS_DEBUG=1 timeout -k 10 300 python -u bench.py --bfs-only > $OUT/bfs_debug.json 2> $OUT/bfs_debug.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_cugraph_api.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bfs" \
  > $OUT/pytest_mg.log 2>&1; rc=$?; tail -1 $OUT/pytest_mg.log; exit $rc

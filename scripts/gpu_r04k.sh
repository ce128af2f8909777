#!/bin/bash
# round-4: BFS claim by the predecessor atomicMin -- tests (incl. RMAT-24 all roots),
# the predecessors' share per root, bench
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04k}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bfs.py "tests/test_gpu_bench_parity.py::test_bfs_rmat24_all_bench_roots" -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_bfs.log 2>&1; rc=$?; tail -2 $OUT/pytest_bfs.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/pytest_bfs.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/bfs_pred_cost.py 24 5 > $OUT/pred_cost.txt 2>&1; rc=$?; grep -E "root|mean" $OUT/pred_cost.txt; [ $rc -eq 0 ] || { tail $OUT/pred_cost.txt; exit $rc; }
TAG=${TAG:-r04k}/bfs MODES="- -" bash scripts/gpu_bfs_ab.sh || exit $?

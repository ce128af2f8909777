#!/bin/bash
# round-4: speculative second bottom-up level -- BFS tests, MG==SG, bench, level log
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04n}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bfs.py "tests/test_gpu_bench_parity.py::test_bfs_rmat24_all_bench_roots" -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_bfs.log 2>&1; rc=$?; tail -2 $OUT/pytest_bfs.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_bfs.log | head; exit $rc; }
TAG=${TAG:-r04n}/bfs MODES="- - -" bash scripts/gpu_bfs_ab.sh || exit $?
CGX_BFS_DEBUG=1 timeout -k 10 300 python -u bench.py --bfs-only > $OUT/bfs_debug.json 2> $OUT/bfs_debug.err || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py -m gpu -x -q --timeout 320 --timeout-method thread -k "bfs or equals_sg" \
  > $OUT/pytest_mg.log 2>&1; rc=$?; tail -2 $OUT/pytest_mg.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_mg.log | head; exit $rc; }

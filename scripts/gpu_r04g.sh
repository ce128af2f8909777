#!/bin/bash
# round-4: MG one-rank RMAT-24 after the alltoallv self-copy, BFS with in-place
# external predecessors (tests, bench)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04g}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bfs.py tests/test_capi_c.py tests/test_gpu_cugraph_api.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $OUT/pytest_bfs.log 2>&1; rc=$?; tail -3 $OUT/pytest_bfs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/mg_one_rank.py 24 > $OUT/mg24.txt 2>&1; rc=$?
grep -E "RMAT-|\[|graphs|BFS" $OUT/mg24.txt | grep -v Gloo; [ $rc -eq 0 ] || { tail $OUT/mg24.txt; exit $rc; }
TAG=${TAG:-r04g}/bfs MODES="- -" bash scripts/gpu_bfs_ab.sh || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_mg.py tests/test_gpu_bench_parity.py -m gpu -x -q \
  --timeout 170 --timeout-method thread > $OUT/pytest_mg.log 2>&1; rc=$?; tail -3 $OUT/pytest_mg.log; [ $rc -eq 0 ] || exit $rc

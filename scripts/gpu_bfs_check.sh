#!/bin/bash
# BFS tests (incl. RMAT-24 from the bench roots, MG BFS rehearsals), then the BFS bench twice
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-bfscheck}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bfs.py "tests/test_gpu_bench_parity.py::test_bfs_rmat24_all_bench_roots" tests/test_capi_c.py tests/test_gpu_cugraph_api.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_bfs.log 2>&1; rc=$?; tail -1 $OUT/pytest_bfs.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_bfs.log | head; exit $rc; }
TAG=${TAG:-bfscheck}/bfs MODES="${MODES:-- -}" bash scripts/gpu_bfs_ab.sh

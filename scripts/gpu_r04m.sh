#!/bin/bash
# round-4: after restoring the BFS work-item pointer -- BFS tests (incl. the
# unrenumbered direction-optimising case) and the MG == SG rehearsals
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04m}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_bfs.log 2>&1; rc=$?; tail -2 $OUT/pytest_bfs.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_bfs.log | head; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py -m gpu -x -v --timeout 320 --timeout-method thread -k "equals_sg or dask" \
  > $OUT/pytest_mg.log 2>&1; rc=$?; tail -2 $OUT/pytest_mg.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_mg.log | head; exit $rc; }

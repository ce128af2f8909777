#!/bin/bash
# round-4: chunked MG PageRank (overlapped column reduce-scatters) -- the MG suite
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04o}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_mg.py -m gpu -x -v --timeout 320 --timeout-method thread \
  > $OUT/pytest_mg.log 2>&1; rc=$?; tail -3 $OUT/pytest_mg.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_mg.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/mg_one_rank.py 22 > $OUT/mg22.txt 2>&1; rc=$?; grep -E "RMAT-|\[-" $OUT/mg22.txt; exit $rc

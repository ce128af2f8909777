#!/bin/bash
# spill fixes (item start time / id from LDS, 4-per-thread window apply): PageRank tests, A/B
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03ab; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/pr_ab.py 24 base base CGX_PR_UNIT_W=0 > $OUT/pr24.txt 2>&1; rc=$?; grep RMAT $OUT/pr24.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/pr_ab.py 22 base base > $OUT/pr22.txt 2>&1; rc=$?; grep RMAT $OUT/pr22.txt; exit $rc

#!/bin/bash
# measured-cost (longest-first) single queue for the 4K-window schedule (RMAT-22): tests, A/B
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03ac; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/pr_ab.py 22 base CGX_PR_CALIB=0 base CGX_PR_CALIB=0 > $OUT/pr22.txt 2>&1; rc=$?; grep RMAT $OUT/pr22.txt; exit $rc

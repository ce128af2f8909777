#!/bin/bash
# PageRank change check: test_gpu_pagerank.py (bitwise A/B tests included), then an
# RMAT-24 A/B of the given settings.  usage: TAG=x bash scripts/gpu_pr_check.sh [pr_ab args...]
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-prcheck}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 400 python -u scripts/pr_ab.py 24 "${@:-base}" > $OUT/pr24.txt 2>&1
rc=$?; grep RMAT $OUT/pr24.txt; exit $rc

#!/bin/bash
# 16K-destination windows (CGX_PR_WIN_BITS=14): parity, then RMAT-24 / RMAT-22 A/B
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03m; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pagerank.py -k "window_bits or packed_entries or multi_window" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/pr_ab.py 24 base CGX_PR_WIN_BITS=14 CGX_PR_WIN_BITS=14,CGX_PR_SHARE_DIV=8 CGX_PR_WIN_BITS=14,CGX_PR_SHARE_DIV=2 base > $OUT/pr24.txt 2>&1
rc=$?; cat $OUT/pr24.txt | grep RMAT; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/pr_ab.py 22 base CGX_PR_WIN_BITS=13 CGX_PR_WIN_BITS=14 > $OUT/pr22.txt 2>&1
rc=$?; cat $OUT/pr22.txt | grep RMAT; exit $rc

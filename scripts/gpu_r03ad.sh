#!/bin/bash
# window bits with measured-cost queues: RMAT-22 and RMAT-24 A/B
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03ad; mkdir -p $OUT
timeout -k 10 300 python -u scripts/pr_ab.py 22 base CGX_PR_WIN_BITS=13 CGX_PR_WIN_BITS=14 > $OUT/pr22.txt 2>&1; rc=$?; grep RMAT $OUT/pr22.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/pr_ab.py 24 base CGX_PR_WIN_BITS=13 CGX_PR_SHARE_DIV=8 CGX_PR_SHARE_DIV=2 > $OUT/pr24.txt 2>&1; rc=$?; grep RMAT $OUT/pr24.txt; exit $rc

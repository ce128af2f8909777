#!/bin/bash
# calibration group size A/B (RMAT-24)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03ai; mkdir -p $OUT
timeout -k 10 400 python -u scripts/pr_ab.py 24 base CGX_PR_CALGROUP=8 CGX_PR_CALGROUP=4 CGX_PR_CALGROUP=32 base CGX_PR_CALGROUP=8 > $OUT/pr24.txt 2>&1; rc=$?; grep RMAT $OUT/pr24.txt; exit $rc

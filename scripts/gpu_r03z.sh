#!/bin/bash
# next-item prefetch + two-pass window apply: bitwise tests, A/B, timeline
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03z; mkdir -p $OUT
true

timeout -k 10 200 python -u scripts/pr_timeline.py 24 > $OUT/timeline.txt 2>&1 || { tail -5 $OUT/timeline.txt; exit 1; }
cp /tmp/pr_timeline.csv $OUT/; grep -E "mean span|launch 9:" $OUT/timeline.txt | cut -c1-200
timeout -k 10 300 python -u scripts/pr_ab.py 24 base CGX_PR_CALIB=0 base > $OUT/pr24.txt 2>&1; rc=$?; grep RMAT $OUT/pr24.txt
timeout -k 10 300 python -u scripts/pr_ab.py 22 base CGX_PR_CALIB=0 CGX_PR_WIN_BITS=12 > $OUT/pr22.txt 2>&1; rc=$?; grep RMAT $OUT/pr22.txt; exit $rc

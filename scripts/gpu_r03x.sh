#!/bin/bash
# PageRank push timeline on RMAT-24 (per-item fetch/end times; tail and busy share)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03x; mkdir -p $OUT
timeout -k 10 300 python -u scripts/pr_timeline.py 24 > $OUT/timeline.txt 2>&1
rc=$?; cp /tmp/pr_timeline.csv $OUT/ 2>/dev/null; tail -22 $OUT/timeline.txt; exit $rc

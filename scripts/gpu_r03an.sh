#!/bin/bash
# RMAT-26 PageRank window bits A/B (16K windows: 2 delta bits, jump-heavy in sparse windows)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03an; mkdir -p $OUT
timeout -k 10 500 python -u scripts/pr_ab.py 26 base CGX_PR_WIN_BITS=13 > $OUT/pr26.txt 2>&1; rc=$?; grep RMAT $OUT/pr26.txt; exit $rc

#!/bin/bash
# ablation: the fused apply's cost on the push's critical path (CGX_PR_ABLATE_APPLY=1 skips
# the apply of whole windows -- wrong ranks, timing only)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03af; mkdir -p $OUT
timeout -k 10 300 python -u scripts/pr_ab.py 24 base CGX_PR_ABLATE_APPLY=1 base CGX_PR_ABLATE_APPLY=1 > $OUT/pr24.txt 2>&1; rc=$?; grep RMAT $OUT/pr24.txt; exit $rc

#!/bin/bash
# round-4: PageRank window-share size A/B (CGX_PR_SHARE_DIV) at RMAT-24 and 26
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SCALES="24" SETTINGS="base CGX_PR_SHARE_DIV=2 CGX_PR_SHARE_DIV=8 CGX_PR_SHARE_DIV=16 base CGX_PR_SHARE_DIV=8" TAG=${TAG:-r04p} bash scripts/gpu_ab.sh || exit $?
SCALES="26" SETTINGS="base CGX_PR_SHARE_DIV=8 CGX_PR_SHARE_DIV=16" LIMIT=450 TAG=${TAG:-r04p} bash scripts/gpu_ab.sh || exit $?
SCALES="22" SETTINGS="base CGX_PR_SHARE_DIV=8 base CGX_PR_SHARE_DIV=8" TAG=${TAG:-r04p} bash scripts/gpu_ab.sh || exit $?

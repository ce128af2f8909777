#!/bin/bash
# round-4: MG one-rank diagnosis (which of fused apply / enc / win bits breaks bitwise
# equality), then the jump-mask A/B of the 16K-window push on one box
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04d}; mkdir -p $OUT
for m in "-" "CGX_PR_WIN_BITS=14" "CGX_PR_WIN_BITS=14,CGX_PR_FUSE=0" "CGX_PR_WIN_BITS=14,CGX_PR_ENC=0" "CGX_PR_WIN_BITS=14,CGX_PR_FUSE=0,CGX_PR_ENC=0" "CGX_PR_WIN_BITS=14,CGX_PR_HUB=0"; do
  envs=""; [ "$m" = "-" ] || envs="${m//,/ }"
  env $envs timeout -k 10 200 python -u scripts/mg_one_rank.py 18 > $OUT/mg1_$RANDOM.txt 2>&1
  rc=$?; echo "== $m: $(grep RMAT- $OUT/mg1_*.txt | tail -1 | cut -d: -f2-)"; rm -f $OUT/mg1_*.txt; [ $rc -eq 0 ] || exit $rc
done
SCALES="24" SETTINGS="base CGX_PR_MASK=0 CGX_PR_MASK=1 base CGX_PR_MASK=0 CGX_PR_MASK=1" TAG=${TAG:-r04d} bash scripts/gpu_ab.sh || exit $?
SCALES="26" SETTINGS="base CGX_PR_MASK=0 CGX_PR_MASK=1" LIMIT=400 TAG=${TAG:-r04d} bash scripts/gpu_ab.sh || exit $?

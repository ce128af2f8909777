#!/bin/bash
# round-4: MG one-rank RMAT-24 (schedule print, BFS cross-check, SG 32-bit entries),
# BFS tests after removing the rejected A/B forms, BFS bench
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04f}; mkdir -p $OUT
CGX_PR_DEBUG=1 SG_PACKED0=1 timeout -k 10 400 python -u scripts/mg_one_rank.py 24 > $OUT/mg24.txt 2>&1; rc=$?
grep -E "RMAT-|\[|graphs|BFS|SG 32" $OUT/mg24.txt | grep -v Gloo; [ $rc -eq 0 ] || { tail $OUT/mg24.txt; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_bfs.log 2>&1; rc=$?; tail -3 $OUT/pytest_bfs.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r04f}/bfs MODES="- -" bash scripts/gpu_bfs_ab.sh || exit $?

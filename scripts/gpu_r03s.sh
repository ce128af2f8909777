#!/bin/bash
# world-8 Louvain rehearsal alone (its failure message), then the PageRank file + hub A/B
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03s; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest "tests/test_gpu_mg.py::test_mg_world8_reference_grid[louvain-2]" -x -q --timeout 240 --timeout-method thread --durations=5 > $OUT/louvain8.log 2>&1
rc=$?; tail -3 $OUT/louvain8.log; [ $rc -le 1 ] || exit $rc
TAG=r03s bash scripts/gpu_pr_check.sh base CGX_PR_HUB=0 base CGX_PR_HUB=0

#!/bin/bash
# gather-cost sweep; Louvain SG + MG tests with poisoned allocations (CGX_POISON=1)
# and per-rank phase traces (CGX_LOUVAIN_TRACE=2) to find the intermittent world-8 stall
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03l; mkdir -p $OUT
TAG=r03l bash scripts/gpu_gcost.sh > /dev/null || exit 1
CGX_POISON=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_louvain.py -x -q --timeout 120 --timeout-method thread > $OUT/sg_poison.log 2>&1
rc=$?; tail -3 $OUT/sg_poison.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
CGX_POISON=1 CGX_LOUVAIN_TRACE=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_mg.py -k louvain -v -s --timeout 200 --timeout-method thread > $OUT/mg_poison.log 2>&1
rc=$?; grep -E "PASS|FAIL" $OUT/mg_poison.log | tail -15; exit $rc

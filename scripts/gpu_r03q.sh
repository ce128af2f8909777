#!/bin/bash
# fused push + apply: parity (bitwise vs the separate apply, window bits, packed), then A/B
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03q; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 400 python -u scripts/pr_ab.py 24 base CGX_PR_FUSE=0 base CGX_PR_FUSE=0 > $OUT/pr24.txt 2>&1
rc=$?; grep RMAT $OUT/pr24.txt; exit $rc

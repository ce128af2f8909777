#!/bin/bash
# MG rehearsal file alone, verbose with durations (the world-8 Louvain failure inside the suite)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03t; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_mg.py -v -rA --timeout 240 --timeout-method thread --durations=0 > $OUT/mg.log 2>&1
rc=$?; tail -5 $OUT/mg.log; exit $rc

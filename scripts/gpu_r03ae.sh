#!/bin/bash
# MG PageRank with per-rank measured-cost queues: MG rehearsals + bench --gpus rehearsal
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03ae; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_mg.py tests/test_bench_launch.py -x -q -m gpu --timeout 200 --timeout-method thread -k "pagerank or world8 or gpus4 or dask" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head; exit $rc; }

#!/bin/bash
# round-4: BFS predecessor translation in place vs the finishing pass (same box, kernel
# stats of both), PageRank window bits at RMAT-22
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04h}; mkdir -p $OUT
TAG=${TAG:-r04h}/bfs MODES="- CGX_BFS_PRED_FINISH=1 - CGX_BFS_PRED_FINISH=1" bash scripts/gpu_bfs_ab.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_inplace -o run -- python3 -u bench.py --bfs-only > $OUT/p1.log 2>&1 || exit $?
CGX_BFS_PRED_FINISH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_finish -o run -- python3 -u bench.py --bfs-only > $OUT/p2.log 2>&1 || exit $?
SCALES="22" SETTINGS="base CGX_PR_WIN_BITS=13 CGX_PR_WIN_BITS=14 base" TAG=${TAG:-r04h} bash scripts/gpu_ab.sh || exit $?
find $OUT -name "*kernel_stats.csv" | head
CGX_BFS_DEBUG=1 timeout -k 10 300 python -u bench.py --bfs-only > $OUT/bfs_debug.json 2> $OUT/bfs_debug.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_parity.py -m gpu -x -q -k "mg_one_rank" --timeout 250 \
  --timeout-method thread > $OUT/pytest_mg1.log 2>&1; rc=$?; tail -3 $OUT/pytest_mg1.log; [ $rc -eq 0 ] || exit $rc

#!/bin/bash
# round-4: BFS in-place external predecessors (probe stores deferred one chunk) vs the
# finishing pass, per-level debug log, kernel stats of both (traces deleted: stats only)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04i}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_bfs.log 2>&1; rc=$?; tail -2 $OUT/pytest_bfs.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r04i}/bfs MODES="- CGX_BFS_PRED_FINISH=1 - CGX_BFS_PRED_FINISH=1" bash scripts/gpu_bfs_ab.sh || exit $?
CGX_BFS_DEBUG=1 timeout -k 10 300 python -u bench.py --bfs-only > $OUT/bfs_debug.json 2> $OUT/bfs_debug.err || exit $?
for m in inplace finish; do
  envs=""; [ $m = finish ] && envs="CGX_BFS_PRED_FINISH=1"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run -- python3 -u bench.py --bfs-only > $OUT/p_$m.log 2>&1 || exit $?
  find $OUT/prof_$m -type f ! -name "*stats.csv" -delete
done
du -sh $OUT

#!/bin/bash
# round-4: BFS level-counter publish without the L2 write-back (A/B against the
# system-scope release), BFS tests three times (ordering of the host words)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04r}; mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py "tests/test_gpu_bench_parity.py::test_bfs_rmat24_all_bench_roots" -m gpu -x -q --timeout 200 --timeout-method thread \
    > $OUT/pytest_bfs_$i.log 2>&1; rc=$?; tail -1 $OUT/pytest_bfs_$i.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/pytest_bfs_$i.log | head; exit $rc; }
done
TAG=${TAG:-r04r}/bfs MODES="- CGX_BFS_PUB_FENCE=1 - CGX_BFS_PUB_FENCE=1" bash scripts/gpu_bfs_ab.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_pub -o run -- python3 -u bench.py --bfs-only > $OUT/p.log 2>&1 || exit $?
f=$(find /tmp/prof_pub -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && grep -E "publish|topdown|probe" "$f" | cut -c1-200

#!/bin/bash
# round-4: BFS predecessor forms -- tests, the predecessors' share per root, A/B of
# atomicMin (default) / k_td_pred pass / finish pass, kernel stats of default and pass
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04j}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py tests/test_gpu_pagerank.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $OUT/pytest_bfs.log 2>&1; rc=$?; tail -2 $OUT/pytest_bfs.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/pytest_bfs.log | head; exit $rc; }
timeout -k 10 300 python -u scripts/bfs_pred_cost.py 24 5 > $OUT/pred_cost.txt 2>&1; rc=$?; grep -E "root|mean" $OUT/pred_cost.txt; [ $rc -eq 0 ] || { tail $OUT/pred_cost.txt; exit $rc; }
TAG=${TAG:-r04j}/bfs MODES="- CGX_BFS_TD_PRED=pass CGX_BFS_TD=bitmap CGX_BFS_PRED_FINISH=1 - CGX_BFS_TD_PRED=pass CGX_BFS_TD=bitmap CGX_BFS_PRED_FINISH=1" bash scripts/gpu_bfs_ab.sh || exit $?
for m in default bitmap; do
  envs=""; [ $m = bitmap ] && envs="CGX_BFS_TD=bitmap"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$m -o run -- python3 -u bench.py --bfs-only > $OUT/p_$m.log 2>&1 || exit $?
  f=$(find /tmp/prof_$m -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats_$m.csv
done
ls $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_outw -o run -- python3 -u scripts/outw_time.py 24 ones > $OUT/outw.log 2>&1 || exit $?
grep "RMAT-" $OUT/outw.log; f=$(find /tmp/prof_outw -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats_outw.csv && grep -i "row_sum" $OUT/kernel_stats_outw.csv
timeout -k 10 200 python -u -m pytest tests/test_gpu_pagerank.py -m gpu -x -q -k "out_weight or outw" --timeout 120 --timeout-method thread > $OUT/pytest_outw.log 2>&1; rc=$?; tail -1 $OUT/pytest_outw.log; exit $rc

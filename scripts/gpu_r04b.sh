#!/bin/bash
# round-4 check: PageRank tests (fused variants, out-weight sums), RMAT-26 parity, MG==SG;
# push A/B (masked jumps, fused small windows); a PageRank-only kernel trace
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04b}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py "tests/test_gpu_bench_parity.py::test_louvain_bench_graph_modularity" tests/test_gpu_mg.py -m gpu -v -rf --timeout 300 --timeout-method thread -k "not world8 and not rank_without and not sssp and not personalized" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest.log | head; [ $rc -eq 1 ] || exit $rc; }
SCALES="22" SETTINGS="base CGX_PR_FUSE_SMALL=1 CGX_PR_MASKJ=1 CGX_PR_FUSE_SMALL=1,CGX_PR_MASKJ=1 base" TAG=${TAG:-r04b} bash scripts/gpu_ab.sh || exit $?
SCALES="24 26" SETTINGS="base CGX_PR_MASKJ=1 base CGX_PR_MASKJ=1" TAG=${TAG:-r04b} LIMIT=400 bash scripts/gpu_ab.sh || exit $?
rm -rf /tmp/prof_r04b
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_r04b -o pr -- python3 bench.py --no-bfs --no-louvain --no-traffic --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof.log 2>&1
rc=$?; f=$(find /tmp/prof_r04b -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv; [ $rc -eq 0 ] || exit $rc
# BFS: the paired probe under the BFS tests, then A/B
CGX_BFS_PROBE2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_bfs.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest_bfs_probe2.log 2>&1
rc=$?; tail -1 $OUT/pytest_bfs_probe2.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r04b}/bfs MODES="- CGX_BFS_PROBE2=1 CGX_BFS_TD_CAP=4096 CGX_BFS_PROBE2=1,CGX_BFS_TD_CAP=4096 -" bash scripts/gpu_bfs_ab.sh || exit $?
for sc in 24 26; do timeout -k 10 300 python -u scripts/pr_window_stats.py $sc > $OUT/winstats_$sc.txt 2>&1 || exit $?; cat $OUT/winstats_$sc.txt; done

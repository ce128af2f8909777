#!/bin/bash
# PageRank queue layouts on RMAT-24: entry-dealt XCD queues (CGX_PR_QMODE=xcd, no
# calibration), measured-cost XCD queues (default), measured-cost global queue;
# per-item timelines + A/B times, after the bitwise tests
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03y; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread -k "calibrated or fused or hub" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head; exit $rc; }
for m in CGX_PR_QMODE=xcd base CGX_PR_DEAL=global; do
  timeout -k 10 200 python -u scripts/pr_timeline.py 24 $([ $m = base ] || echo $m) > $OUT/timeline_$m.txt 2>&1 || { tail -5 $OUT/timeline_$m.txt; exit 1; }
  cp /tmp/pr_timeline.csv $OUT/pr_timeline_$m.csv; echo "$m: $(grep 'mean span' $OUT/timeline_$m.txt) $(grep 'launch 9:' $OUT/timeline_$m.txt | cut -c1-150)"
done
timeout -k 10 300 python -u scripts/pr_ab.py 24 base CGX_PR_QMODE=xcd CGX_PR_DEAL=global base CGX_PR_QMODE=xcd > $OUT/pr24.txt 2>&1; rc=$?; grep RMAT $OUT/pr24.txt; exit $rc

#!/bin/bash
# round 3 step i: source-dedup push A/B + bitwise tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pagerank.py -k "dedup or packed or encoded" -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/pr_ab.py 24 base CGX_PR_DEDUP=1 base CGX_PR_DEDUP=1 > $O/pr24.txt 2>&1 || { tail $O/pr24.txt; exit 1; }
cat $O/pr24.txt
timeout -k 10 200 python -u scripts/pr_ab.py 22 base CGX_PR_DEDUP=1 > $O/pr22.txt 2>&1 || { tail $O/pr22.txt; exit 1; }
cat $O/pr22.txt
echo ALLDONE

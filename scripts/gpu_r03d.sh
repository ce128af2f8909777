#!/bin/bash
# round 3 step d: PageRank source slices (tests + A/B + ablations), BFS tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_bfs.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u scripts/pr_ab.py 24 base CGX_PR_SLICE=0 CGX_PR_ABLATE=1 CGX_PR_ABLATE=2 CGX_PR_SLICE=0,CGX_PR_ABLATE=1 CGX_PR_SLICE=0,CGX_PR_ABLATE=2 CGX_PR_SLICE=0,CGX_PR_ABLATE=3,CGX_PR_ABLATE_XMASK=0xFFFF CGX_PR_SLICE_HEAD=131072 CGX_PR_SLICE_SRC=393216 base > $O/pr24.txt 2>&1 || { tail $O/pr24.txt; exit 1; }
cat $O/pr24.txt
timeout -k 10 200 python -u scripts/pr_ab.py 22 base CGX_PR_SLICE=0 CGX_PR_SLICE_HEAD=131072 > $O/pr22.txt 2>&1 || { tail $O/pr22.txt; exit 1; }
cat $O/pr22.txt
echo ALLDONE

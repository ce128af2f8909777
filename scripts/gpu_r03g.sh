#!/bin/bash
# round 3 step g: software-pipelined push (two units' gathers in flight)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/pr_ab.py 24 base base > $O/pr24.txt 2>&1 || { tail $O/pr24.txt; exit 1; }
cat $O/pr24.txt
timeout -k 10 200 python -u scripts/pr_ab.py 22 base > $O/pr22.txt 2>&1 || { tail $O/pr22.txt; exit 1; }
cat $O/pr22.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_bench_parity.py -m gpu -x -v --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo ALLDONE

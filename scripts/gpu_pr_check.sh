set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04v
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04v/pytest_pr.log 2>&1; rc=$?; tail -2 gpurun_out/r04v/pytest_pr.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r04v/pytest_pr.log | head; exit $rc; }
SCALES="22" SETTINGS="base pr_win_bits=12 base" TAG=r04v bash scripts/gpu_ab.sh

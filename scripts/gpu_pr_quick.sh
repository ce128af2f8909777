set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_pr.log 2>&1; rc=$?; tail -3 gpurun_out/pt_pr.log; [ $rc -eq 0 ] || exit $rc
MODES="${MODES:-0 1 2}" bash scripts/ablate.sh 2>&1 | tee gpurun_out/ablate.log

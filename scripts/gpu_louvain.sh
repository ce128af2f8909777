set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_louvain.py tests/test_gpu_mg.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_lv.log 2>&1; rc=$?; tail -25 gpurun_out/pt_lv.log; exit $rc

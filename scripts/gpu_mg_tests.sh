set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_mg.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_mg.log 2>&1; rc=$?; grep -v Gloo gpurun_out/pt_mg.log | grep "Error\|assert\|passed\|failed\|^E " | tail -20; [ $rc -eq 0 ] || exit $rc
N=4 bash scripts/gpu_mg_rehearsal.sh

mkdir -p gpurun_out/r04t
timeout -k 10 500 python -u -m pytest tests/test_gpu_mg.py -m gpu -x -q -s --timeout 300 --timeout-method thread -k "louvain or equals_sg" > gpurun_out/r04t/mg.log 2>&1; rc=$?
grep -E "MG Louvain|RMAT-1|passed|failed" gpurun_out/r04t/mg.log; exit $rc

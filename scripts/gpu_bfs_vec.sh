# BFS vector-probe check: BFS tests, the RMAT-24 bench-parity test with CGX_BFS_PROBE_VEC=1, then A/B
set -o pipefail
OUT=gpurun_out/${TAG:-bfsvec}; mkdir -p $OUT
CGX_BFS_PROBE_VEC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k bfs > $OUT/pytest_vec.log 2>&1
rc=$?; tail -2 $OUT/pytest_vec.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-bfsvec} TESTS="tests/test_gpu_bfs.py" MODES="${MODES:-- CGX_BFS_PROBE_VEC=1 - CGX_BFS_PROBE_VEC=1}" bash scripts/gpu_bfs_ab.sh

set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=r02c_tr CHILD="--traffic-child bfs --bfs-scale 24 --bfs-roots 8" bash scripts/gpu_trace.sh || exit $?
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; grep "\[bench\]" $OUT/bench.err; exit $rc

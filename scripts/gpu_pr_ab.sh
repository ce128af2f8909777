# PageRank A/B: tests, then the bench's PageRank legs under each CGX_PR_WIN_BITS setting
set -o pipefail
OUT=gpurun_out/${TAG:-prab}; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_bench_parity.py -x -v --timeout 300 --timeout-method thread -k "${TESTS_K:-.}" > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; grep -E "RMAT-.*iterations" $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for wb in ${WBS:-default 12 13}; do
  if [ $wb = default ]; then unset CGX_PR_WIN_BITS; else export CGX_PR_WIN_BITS=$wb; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-louvain --no-bfs --no-traffic --steps 5 > $OUT/bench_$wb.json 2> $OUT/bench_$wb.err
  rc=$?; echo "== win bits $wb"; grep "edges/s" $OUT/bench_$wb.err; [ $rc -eq 0 ] || { tail $OUT/bench_$wb.err; exit $rc; }
done

# tests for the given files, then the default bench (no CPU baselines, no PMC passes)
set -o pipefail
OUT=gpurun_out/${TAG:-quick}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-traffic ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; grep "\[bench\]" $OUT/bench.err; [ $rc -eq 0 ] || { tail $OUT/bench.err; exit $rc; }

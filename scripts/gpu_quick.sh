#!/bin/bash
# One GPU call: named test selections, then optional bench; each step under its own limit.
# usage: TAG=r05a TESTS="tests/a.py::t tests/b.py" BENCH=1 bash scripts/gpu_quick.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
if [ -n "${PRE:-}" ]; then
  timeout -k 10 300 bash -c "$PRE" > $OUT/pre.log 2>&1; rc=$?; tail -30 $OUT/pre.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${TESTS:-}" ]; then
  CGX_TEST_CLOCK=1 timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -v -rf ${PYTEST_EXTRA:-} --timeout 400 --timeout-method thread --durations=20 > $OUT/pytest.log 2>&1
  rc=$?; tail -25 $OUT/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 600 python -u bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; grep "\[bench\]" $OUT/bench.err; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
fi

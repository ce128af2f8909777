# One GPU call: pytest -m gpu, the default bench line, and a rocprofv3 kernel-trace
# profile of the bench (kernel stats), each step under its own time limit.
# usage: TAG=r02a bash scripts/gpu_round.sh [skip-tests]
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${1:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; grep "\[bench\]" $OUT/bench.err; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o bench -- python3 bench.py --no-traffic --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?
f=$(find /tmp/prof_$TAG -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv
f=$(find /tmp/prof_$TAG -name "*kernel_trace.csv" | head -1); [ -n "$f" ] && gzip -c "$f" > $OUT/kernel_trace.csv.gz
exit $rc

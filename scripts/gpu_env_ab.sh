# Generic A/B: optional tests, then the bench's PageRank legs under each MODES entry
# (space-separated env assignments joined by ',', "-" = defaults), alternating
set -o pipefail
OUT=gpurun_out/${TAG:-envab}; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; grep -E "RMAT-.*iterations|FAILED" $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for m in ${MODES:-- -}; do
  i=$((i+1)); envs=""; [ "$m" = "-" ] || envs="${m//,/ }"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-louvain --no-bfs --no-traffic --steps ${STEPS:-5} ${BENCH_ARGS:-} > $OUT/b_$i.json 2> $OUT/b_$i.err
  rc=$?; echo "== $m"; grep -E "edges/s|ms/iter" $OUT/b_$i.err | head -4; [ $rc -eq 0 ] || { tail $OUT/b_$i.err; exit $rc; }
done

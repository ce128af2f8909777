# BFS A/B: optional tests, then bench.py --bfs-only under each MODES entry
# (env assignments joined by ',', "-" = defaults)
set -o pipefail
OUT=gpurun_out/${TAG:-bfsab}; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; grep -E "FAILED" $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for m in ${MODES:-- -}; do
  i=$((i+1)); envs=""; [ "$m" = "-" ] || envs="${m//,/ }"
  env $envs timeout -k 10 300 python -u bench.py --bfs-only ${BENCH_ARGS:-} > $OUT/b_$i.json 2> $OUT/b_$i.err
  rc=$?; echo "== $m: $(grep '\[bench\]' $OUT/b_$i.err)"; [ $rc -eq 0 ] || { tail $OUT/b_$i.err; exit $rc; }
done

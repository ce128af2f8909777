# Louvain A/B: the Louvain tests, then the bench Louvain leg under each setting of
# MODES (space-separated env assignments, "-" = defaults), traced per sweep
set -o pipefail
OUT=gpurun_out/${TAG:-lv}; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_louvain.py} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
fi
i=0
for m in ${MODES:-- CGX_LOUVAIN_HASH=0 -}; do
  i=$((i+1)); envs=""; [ "$m" = "-" ] || envs="$m"
  env $envs CGX_LOUVAIN_TRACE=1 timeout -k 10 300 python -u bench.py --louvain-only ${BENCH_ARGS:-} > $OUT/lv_$i.json 2> $OUT/lv_$i.err
  rc=$?; echo "$m: $(grep '\[bench\]' $OUT/lv_$i.err)"; [ $rc -eq 0 ] || { tail $OUT/lv_$i.err; exit $rc; }
done

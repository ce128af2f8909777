# same-box A/B of library builds on the bench's PageRank legs: LIBS="name=path ..."
set -o pipefail
OUT=gpurun_out/${TAG:-libab}; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for spec in $LIBS; do
    name=${spec%%=*}; path=${spec#*=}
    if [ "$path" = default ]; then unset CUGRAPH_AMD_LIB; else export CUGRAPH_AMD_LIB=$PWD/$path; fi
    timeout -k 10 300 env $EXTRA python -u bench.py ${BENCH_AB_ARGS:---no-cpu-baseline --no-louvain --no-bfs --no-traffic --steps 5} > $OUT/b_${name}_$rep.json 2> $OUT/b_${name}_$rep.err
    rc=$?; echo "== $name rep $rep"; grep "\[bench\].*/s\|MTEPS" $OUT/b_${name}_$rep.err; [ $rc -eq 0 ] || { tail $OUT/b_${name}_$rep.err; exit $rc; }
  done
done

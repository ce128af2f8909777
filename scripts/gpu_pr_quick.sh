# PageRank tests + PageRank-only bench pairs under MODES (env assignments joined by ',', "-" = defaults)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prq}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_pagerank.py} -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS_K:-not louvain}" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in ${MODES:-- -}; do
  envs=""; [ "$m" = "-" ] || envs="${m//,/ }"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-louvain --no-bfs --no-traffic --steps 5 > $OUT/b.json 2> $OUT/b.err
  rc=$?; echo "== $m"; grep "edges/s" $OUT/b.err; [ $rc -eq 0 ] || { tail $OUT/b.err; exit $rc; }
done

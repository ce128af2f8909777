# Round-2 A/B: PageRank encoded x~ (CGX_PR_ENC) and BFS host-path changes, after
# the PageRank/BFS GPU tests.  usage: TAG=... bash scripts/gpu_ab_r02d.sh
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02d}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_pagerank.py tests/test_gpu_bfs.py tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTS_K:-not louvain}" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in ${MODES:-CGX_PR_ENC=0 - CGX_PR_ENC=0 -}; do
  envs=""; [ "$m" = "-" ] || envs="${m//,/ }"
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-louvain --no-traffic --steps 5 > $OUT/b.json 2> $OUT/b.err
  rc=$?; echo "== $m"; grep "edges/s\|MTEPS" $OUT/b.err; [ $rc -eq 0 ] || { tail $OUT/b.err; exit $rc; }
done

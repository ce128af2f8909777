#!/bin/bash
# BFS A/B: optional tests, then bench.py --bfs-only under each MODES entry (handle
# options name=value joined by ',', "-" = defaults), the modes interleaved ROUNDS times
# usage: TAG=r05ab MODES="- bfs_prefetch_off=0" ROUNDS=2 bash scripts/gpu_bfs_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-bfsab}; mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; grep -E "FAILED" $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for r in $(seq ${ROUNDS:-1}); do
  for m in ${MODES:-- -}; do
    i=$((i+1)); opts=""; [ "$m" = "-" ] || opts="$m"
    timeout -k 10 300 python -u bench.py --bfs-only --options "$opts" ${BENCH_ARGS:-} > $OUT/b_$i.json 2> $OUT/b_$i.err
    rc=$?; echo "== $m: $(grep '\[bench\]' $OUT/b_$i.err)" | tee -a $OUT/ab.log; [ $rc -eq 0 ] || { tail $OUT/b_$i.err; exit $rc; }
  done
done

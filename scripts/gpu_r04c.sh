#!/bin/bash
# round-4: push with masked jump lanes (tests + PageRank-only bench with traffic), one-rank
# RCCL MG vs SG at RMAT-24, and the world-8 Louvain rehearsal with SDMA copies enabled
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04c}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_pagerank.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest_pr.log 2>&1
rc=$?; tail -1 $OUT/pytest_pr.log; [ $rc -eq 0 ] || { grep FAILED $OUT/pytest_pr.log; exit $rc; }
timeout -k 10 500 python -u bench.py --no-bfs --no-louvain --no-cpu-baseline --steps 5 > $OUT/bench_pr.json 2> $OUT/bench_pr.err
rc=$?; grep "\[bench\]" $OUT/bench_pr.err; [ $rc -eq 0 ] || { tail $OUT/bench_pr.err; exit $rc; }
timeout -k 10 300 python -u scripts/mg_one_rank.py 24 > $OUT/mg_one_rank.txt 2>&1
rc=$?; cat $OUT/mg_one_rank.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  HSA_ENABLE_SDMA=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mg.py -m gpu -v --timeout 250 --timeout-method thread -k "world8 and louvain" > $OUT/hang_$i.log 2>&1
  rc=$?; echo "world-8 Louvain with SDMA, run $i: rc $rc"; tail -1 $OUT/hang_$i.log; [ $rc -eq 0 ] || exit $rc
done

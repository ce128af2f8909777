#!/bin/bash
# round-4: MG one-rank RMAT-24 diagnosis by switch, the add-only jump mask default on
# the bench scales, the new GPU tests, then the default bench (row sums, first call)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04e}; mkdir -p $OUT
timeout -k 10 150 python -u -m pytest tests/test_gpu_mg.py::test_mg_louvain_negative_weight_refused \
  tests/test_gpu_pagerank.py::test_out_weight_sums_tiled -m gpu -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/mg_one_rank.py 24 - CGX_PR_FUSE=0 CGX_PR_HUB=0 CGX_PR_ENC=0 \
  CGX_PR_FUSE=0,CGX_PR_HUB=0,CGX_PR_ENC=0 > $OUT/mg24.txt 2>&1; rc=$?; grep -E "RMAT-|\[" $OUT/mg24.txt | grep -v Gloo; [ $rc -eq 0 ] || { tail $OUT/mg24.txt; exit $rc; }
CGX_PR_CALIB=0 timeout -k 10 300 python -u scripts/mg_one_rank.py 24 > $OUT/mg24c.txt 2>&1; rc=$?; echo "CALIB=0:"; grep -E "RMAT-|\[-" $OUT/mg24c.txt; [ $rc -eq 0 ] || { tail $OUT/mg24c.txt; exit $rc; }
timeout -k 10 300 python -u scripts/mg_one_rank.py 22 > $OUT/mg22.txt 2>&1; rc=$?; grep -E "RMAT-|\[-" $OUT/mg22.txt; [ $rc -eq 0 ] || { tail $OUT/mg22.txt; exit $rc; }
SCALES="22 24" SETTINGS="base base" TAG=${TAG:-r04e} bash scripts/gpu_ab.sh || exit $?
timeout -k 10 600 python -u bench.py --no-traffic > $OUT/bench.json 2> $OUT/bench.err; rc=$?
grep "\[bench\]" $OUT/bench.err; [ $rc -eq 0 ] || { tail $OUT/bench.err; exit $rc; }

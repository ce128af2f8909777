#!/bin/bash
# why the world-8 rehearsals crawl inside the full suite: bench-parity module first,
# then one world-8 rehearsal, sampling the busiest threads every 10 s
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03v; mkdir -p $OUT
env | grep -E "OMP|GOMP|KMP|MAX_JOBS|NUM_THREADS" > $OUT/env.txt
nproc >> $OUT/env.txt; grep -c processor /proc/cpuinfo >> $OUT/env.txt; cat /sys/fs/cgroup/cpu.max >> $OUT/env.txt 2>/dev/null
( for i in $(seq 1 40); do sleep 10; echo "--- $i"; top -b -n1 -H | head -30; done ) > $OUT/ps.txt 2>&1 &
SAMPLER=$!
CGX_TEST_CLOCK=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_parity.py "tests/test_gpu_mg.py::test_mg_world8_reference_grid[pagerank-2]" "tests/test_gpu_mg.py::test_mg_world8_reference_grid[louvain-2]" -v --timeout 300 --timeout-method thread --durations=10 > $OUT/pytest.log 2>&1
rc=$?
kill $SAMPLER
tail -15 $OUT/pytest.log
exit $rc

#!/bin/bash
# One GPU call: kernel + memory-copy trace of one-rank RCCL MG BFS and SG BFS at
# RMAT-24 from the bench's 8 roots (scripts/mg_bfs_ab.py), for the per-kernel table.
# usage: TAG=r06f SCALE=24 bash scripts/gpu_mg_bfs_trace.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-mgbfs}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/mg_bfs_ab.py ${SCALE:-24} 40,64 > $OUT/ab.txt 2>&1
rc=$?; tail -4 $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/prof_mgbfs -o mgbfs -- python3 scripts/mg_bfs_ab.py ${SCALE:-24} 40,64 > $OUT/prof.log 2>&1
rc=$?
for f in $(find /tmp/prof_mgbfs -name "*kernel_trace.csv" -o -name "*memory_copy_trace.csv"); do cp "$f" $OUT/; done
exit $rc

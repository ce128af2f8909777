#!/bin/bash
# First PageRank call on a fresh graph: wall times, then a kernel trace of the same.
# usage: TAG=r05d bash scripts/gpu_first_call.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-first}; mkdir -p $OUT
timeout -k 10 200 python3 -u scripts/pr_first_call.py 24 3 > $OUT/first.log 2>&1 || exit $?
cat $OUT/first.log
rm -rf /tmp/prof_first
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_first -o run -- python3 -u scripts/pr_first_call.py 24 1 > $OUT/prof.log 2>&1 || exit $?
f=$(find /tmp/prof_first -name "*kernel_trace.csv" | head -1); [ -n "$f" ] && gzip -c "$f" > $OUT/first_trace.csv.gz
echo done

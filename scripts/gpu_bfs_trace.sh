#!/bin/bash
# BFS leg (bench.py --bfs-only, RMAT-24, 8 roots) under rocprofv3 --kernel-trace: the
# gzipped trace for scripts/bfs_timeline.py and the kernel stats.
# usage: TAG=r05m bash scripts/gpu_bfs_trace.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-bfstrace}; mkdir -p $OUT
rm -rf /tmp/prof_bfst
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bfst -o run -- python3 -u bench.py --bfs-only --no-traffic ${BFS_ARGS:-} > $OUT/p.log 2>&1 || exit $?
f=$(find /tmp/prof_bfst -name "*kernel_trace.csv" | head -1); [ -n "$f" ] && mkdir -p $OUT/kt && cp "$f" $OUT/kt/ && gzip -f $OUT/kt/*.csv
f=$(find /tmp/prof_bfst -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv
grep "\[bench\]" $OUT/p.log

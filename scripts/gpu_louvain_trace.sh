#!/bin/bash
# Louvain leg (bench.py --louvain-only, RMAT-23) under rocprofv3 --kernel-trace: the
# kernel trace (gzipped) and stats for scripts/trace_window.py-style analysis.
# usage: TAG=r05c bash scripts/gpu_louvain_trace.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-lvtrace}; mkdir -p $OUT
rm -rf /tmp/prof_lvt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_lvt -o run -- python3 -u bench.py --louvain-only ${LV_ARGS:-} > $OUT/p.log 2>&1 || exit $?
f=$(find /tmp/prof_lvt -name "*kernel_trace.csv" | head -1); [ -n "$f" ] && gzip -c "$f" > $OUT/louvain_trace.csv.gz
f=$(find /tmp/prof_lvt -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv
grep "\[bench\]" $OUT/p.log

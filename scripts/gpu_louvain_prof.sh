#!/bin/bash
# Louvain leg under rocprofv3 (kernel stats), plus CGX_LOUVAIN_TRACE per-sweep log
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-lvprof}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_lv -o run -- python3 -u bench.py --louvain-only > $OUT/p.log 2>&1 || exit $?
f=$(find /tmp/prof_lv -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/kernel_stats.csv
CGX_LOUVAIN_TRACE=1 timeout -k 10 300 python3 -u bench.py --louvain-only > $OUT/trace.json 2> $OUT/trace.err || exit $?
grep -c "" $OUT/trace.err

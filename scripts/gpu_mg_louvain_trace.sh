#!/bin/bash
# One-rank MG Louvain beside SG (scripts/mg_louvain_once.py) under rocprofv3 --kernel-trace.
# usage: TAG=r05at SCALE=23 bash scripts/gpu_mg_louvain_trace.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-mglvt}; mkdir -p $OUT
rm -rf /tmp/prof_mglv
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_mglv -o run -- python3 -u scripts/mg_louvain_once.py ${SCALE:-23} 2 > $OUT/p.log 2>&1 || { tail -20 $OUT/p.log; exit 1; }
f=$(find /tmp/prof_mglv -name "*kernel_trace.csv" | head -1); [ -n "$f" ] && gzip -c "$f" > $OUT/trace.csv.gz
grep call $OUT/p.log

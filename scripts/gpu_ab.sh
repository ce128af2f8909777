#!/bin/bash
# PageRank A/B on the bench graphs (scripts/pr_ab.py: one resident graph per setting,
# 16 iterations per call, HIP-event ms per iteration), each scale under its own limit.
# usage: TAG=r04b SCALES="22 24" SETTINGS="base pr_hub=0" bash scripts/gpu_ab.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for sc in ${SCALES:-24}; do
  timeout -k 10 ${LIMIT:-300} python -u scripts/pr_ab.py $sc ${SETTINGS:-base} >> $OUT/ab.log 2> $OUT/ab_$sc.err
  rc=$?; tail -n 20 $OUT/ab.log | grep "RMAT-$sc"; [ $rc -eq 0 ] || { tail $OUT/ab_$sc.err; exit $rc; }
done

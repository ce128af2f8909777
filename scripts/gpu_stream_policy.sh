#!/bin/bash
# Does the cache policy of a read-once 16-B stream keep a small gather table in the
# L2 (the push's entry stream beside its x~ gathers)?  Table 3 MB (fits an XCD's
# 4 MB L2), stream 1.5 GB; time per policy, then TCC_HIT / TCC_MISS per policy.
# usage: TAG=r05s bash scripts/gpu_stream_policy.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-spol}; mkdir -p $OUT
B=scripts/ubench/mem_calib
for tmb in 3 6; do
  for aux in 0 2 1 16 17 3 18 19; do
    REPS=5 timeout -k 5 60 $B streamgather $tmb 1536 8192 $aux >> $OUT/time.txt 2>&1 || exit $?
  done
done
cat $OUT/time.txt
for aux in 0 2 16 19; do
  d=/tmp/spmc_${aux}
  REPS=2 timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $d -o run --output-format csv -- $B streamgather 3 1536 8192 $aux > /dev/null 2>&1 || exit $?
  f=$(find $d -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$aux" <<'PY' >> $OUT/pmc.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("aux", sys.argv[2], {k: f"{sorted(v)[len(v)//2]:.4g}" for k, v in agg.items()}, "launches", max(len(v) for v in agg.values()))
PY
done
cat $OUT/pmc.txt

#!/bin/bash
# Random 4-B gathers from a 35 MB table (the RMAT-24 x~) by cache policy: time, and
# per policy the fabric requests (TCC_EA0_RDREQ / _32B) and FETCH_SIZE, one --pmc pass
# each.  usage: TAG=r05g bash scripts/gpu_gather_policy.sh
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-gpol}; mkdir -p $OUT
B=scripts/ubench/mem_calib
for aux in 0 2 1 16 17 3 18 19; do
  REPS=5 timeout -k 5 60 $B gatherk 35 200 8192 $aux >> $OUT/time.txt 2>&1 || exit $?
done
cat $OUT/time.txt
for aux in 0 2 16 17 19; do
  for ctr in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "FETCH_SIZE"; do
    d=/tmp/pmc_${aux}_${ctr%% *}
    REPS=2 timeout -s KILL 60 rocprofv3 --pmc $ctr -d $d -o run --output-format csv -- $B gatherk 35 200 8192 $aux > /dev/null 2>&1 || exit $?
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
done
cat $OUT/pmc.txt

#!/bin/bash
# Memory calibration on the GPU box (scripts/ubench/mem_calib.hip): copy-ceiling sweep
# and the FETCH_SIZE / request-size calibration of random 4-B gathers.  Output under
# gpurun_out/calib/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/calib
mkdir -p $O
B=./scripts/ubench/mem_calib
export TMPDIR=/tmp
{
  for blk in 256 512 1024; do
    for u in 1 2 4 8; do
      for g in 1024 2048 4096 8192; do
        timeout -k 5 30 $B copy 4096 $blk $u $g 1 || exit 1
      done
    done
  done
  for u in 2 4 8; do timeout -k 5 30 $B copy 4096 256 $u 65536 0 || exit 1; done
  for u in 2 4 8; do timeout -k 5 30 $B copy 4096 256 $u 1048576 1 || exit 1; done
  for u in 4 8 16; do
    for g in 2048 4096 8192; do timeout -k 5 30 $B read 4096 256 $u $g || exit 1; done
  done
  for t in 4 35 140 300 1024; do timeout -k 5 60 $B gather $t 200 8192 || exit 1; done
} > $O/sweep.txt 2>&1 || exit 1
timeout -k 5 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
cd /tmp
for ctr in FETCH_SIZE TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_REQ_sum TCC_MISS_sum; do
  for run in "gather 300 200 8192" "gather 35 200 8192" "gather 4 200 8192" "read 1024 256 8 4096" "copy 1024 256 4 4096 1"; do
    tag=$(echo "$ctr $run" | tr ' ' '_')
    REPS=3 timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d /tmp/pmc_$tag -o pmc -- \
      "$GRAFT_REPO_ROOT/scripts/ubench/mem_calib" $run > /dev/null 2>&1 || { echo "$tag failed" >> "$GRAFT_REPO_ROOT/$O/pmc.txt"; continue; }
    f=$(find /tmp/pmc_$tag -name '*counter_collection.csv' | head -1)
    python3 - "$f" "$tag" >> "$GRAFT_REPO_ROOT/$O/pmc.txt" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
vals = [float(r["Counter_Value"]) for r in rows]
print(sys.argv[2], "launches", len(vals), "per-launch", [round(v) for v in vals[-3:]])
EOF
  done
done
echo done >> "$GRAFT_REPO_ROOT/$O/pmc.txt"

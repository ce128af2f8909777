#!/bin/bash
# gather-instruction cost sweep (scripts/ubench/gather_cost.hip)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-gcost}; mkdir -p $OUT
B=scripts/ubench/gather_cost
for kb in 16 2048 262144; do
  for L in 0 1 2 4 8 16 32 64; do
    timeout -k 5 30 $B $kb $L 64 >> $OUT/gcost.txt || exit 1
  done
  for k in 1 4 16 32; do
    timeout -k 5 30 $B $kb 64 $k >> $OUT/gcost.txt || exit 1
    timeout -k 5 30 $B $kb 4 $k >> $OUT/gcost.txt || exit 1
  done
done
cat $OUT/gcost.txt

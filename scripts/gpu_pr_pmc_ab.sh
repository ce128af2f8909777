#!/bin/bash
# HBM bytes and L2 hits/misses of the PageRank push per launch for each handle-option
# setting (pr_ab.py 24 <setting>): FETCH_SIZE, WRITE_SIZE, TCC_HIT/MISS, one pass each.
# usage: TAG=r05h SETTINGS="base pr_band_cut=1048576" bash scripts/gpu_pr_pmc_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-prpmcab}; mkdir -p $O
export TMPDIR=/tmp
for st in ${SETTINGS:-base}; do
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
    i=$((i+1)); rm -rf /tmp/pab$i
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d /tmp/pab$i -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/pr_ab.py ${SCALE:-24} $st > $GRAFT_REPO_ROOT/$O/pab_${st}_$i.log 2>&1) || { echo "pmc $st $i failed"; tail -5 $O/pab_${st}_$i.log; exit 1; }
    echo "== $st" >> $O/pmc.txt
    python3 scripts/pmc_push.py /tmp/pab$i >> $O/pmc.txt
  done
done
cat $O/pmc.txt

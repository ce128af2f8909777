#!/bin/bash
# round 3 step h: TA / TD / TCP counters of the push (is the texture path the bound?)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03h; mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
           "TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_LFIFO_STALL_CYCLES_sum TCP_RFIFO_STALL_CYCLES_sum TCP_TCP_LATENCY_sum"; do
  i=$((i+1)); rm -rf /tmp/pmc$i
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc$i -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/pr_ab.py 24 base > $GRAFT_REPO_ROOT/$O/pmc$i.log 2>&1) || { echo "pmc $i failed"; tail -5 $O/pmc$i.log; continue; }
  python3 scripts/pmc_push.py /tmp/pmc$i >> $O/pmc.txt
  echo "pmc set $i done"
done
cat $O/pmc.txt
echo ALLDONE

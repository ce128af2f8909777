#!/bin/bash
# PMC passes of the PageRank push on RMAT-24 (pr_ab.py, 2 warm + 5 timed calls): wave states,
# instruction mix, texture path, L1->L2 requests, HBM bytes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-prpmc}; mkdir -p $O
export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1)); rm -rf /tmp/pmc$i
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc$i -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/pr_ab.py 24 base > $GRAFT_REPO_ROOT/$O/pmc$i.log 2>&1) || { echo "pmc $i failed"; tail -5 $O/pmc$i.log; exit 1; }
  python3 scripts/pmc_push.py /tmp/pmc$i >> $O/pmc.txt
  echo "pmc set $i done"
done
cat $O/pmc.txt
